# Attention kernel variants (development knobs in csrc/attention.hip), kernel-trace stats each.
export TMPDIR=/tmp
OUT=gpurun_out/attnvar
mkdir -p $OUT
run() {  # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- python3 tools/attn_pmc.py 20 > $OUT/$name.log 2>&1 || return 1
  echo "== $name $*"; python3 tools/kstats.py $OUT/$name/run_kernel_stats.csv 23 | grep attn_
}
run base PK_NOOP=1 && run occ4 PK_ATTN_DKV_OCC=4 && run pad24k PK_ATTN_LDS_PAD=24576 && run pad40k PK_ATTN_LDS_PAD=40960 && run occ4pad PK_ATTN_DKV_OCC=4 PK_ATTN_LDS_PAD=20000
