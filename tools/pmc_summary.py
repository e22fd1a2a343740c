"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, one counter per pass, as
MI355X_MICROARCH.md's rocprofv3 section requires) into per-kernel-family HBM traffic per
launch.

  python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json> [bench.json]

With bench.json (the JSON line of the same `bench.py --eager --warmup 0` command the passes
profiled), a family listed in PER_ENTRY is reported per ENTRY-POINT call: its kernels' bytes
over every dispatch / the calls the bench's probe counted for that entry point (one entry call
may launch several kernels). pk_linear_ex is such a family: every per-point layer launch of the
step goes through it (ops.linear_fwd included), so its bytes match bench.py's roofline unit.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is in KiB and on gfx950
reports half the bytes of 16-B-per-lane coalesced reads, so it is doubled; WRITE_SIZE
(KiB) is exact for 16-B-per-lane stores. Both are L2 memory-side request counters,
with Infinity-Cache hits counted, so this is an upper bound on HBM bytes.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# libposekern entry point -> device kernels it launches (substring match on the name)
FAMILIES = {
    "pk_fps": ["fps_pruned_kernel", "fps_kernel"],
    "pk_sor": ["sor_knn_kernel", "sor_stats_kernel", "sor_count_kernel", "sor_write_kernel"],
    "pk_ball_query_mask": ["bq_mask_stream_kernel", "bq_mask_f32_kernel"],
    "pk_backproject": ["bp_count_kernel", "bp_write_kernel"],
    "pk_spectral_diffusion": ["spec_reduce_mfma_kernel", "spec_combine4_kernel", "spec_expand_mfma_kernel",
                              "spec_reduce_kernel", "spec_combine_kernel", "spec_expand_kernel"],
    "pk_attention_fwd": ["attn_fwd_kernel"],
    "pk_attention_bwd": ["attn_bwd_kernel", "attn_bwd_dq_reduce_kernel"],
    "pk_linear_wgrad": ["wgrad_v2_kernel", "wgrad_partial_kernel", "wgrad_reduce_kernel"],
    "pk_feat_dist_topk": ["fd_top1_prep_kernel", "fd_top1_kernel", "fd_top1_merge_kernel", "fd_prep_kernel",
                          "fd_main_direct_kernel", "fd_merge_kernel"],
    "pk_cgt_lstsq": ["cgt_count_kernel", "cgt_partial_kernel", "cgt_reduce_kernel", "cgt_solve_kernel"],
    # pk_linear_fwd and pk_linear_ex (its epilogue / placement variant) launch the same kernels: the
    # counters cannot tell them apart, so they form one family, per KERNEL launch
    "pk_linear_fwd+ex": ["linear_glds_rows_kernel", "linear_fwd_rows_kernel", "linear_fwd_cf_kernel", "linear_fwd_kernel",
                         "linear_thin_kernel", "linear_cf_pair_kernel"],
    "pk_linear_wgrad_grouped": ["wgrad_glds_grouped_kernel", "wgrad_grouped_kernel", "wgrad_grouped_reduce_kernel"],
    "pk_nce_loss": ["nce_pass_kernel<false>", "nce_pass_kernel<true>", "nce_scatter_kernel"],
    "pk_clip_rmsprop": ["grad_sumsq_kernel", "clip_rmsprop_kernel"],
    "pk_instnorm_relu_fwd": ["instnorm_relu_fwd"],
    "pk_instnorm_relu_bwd": ["instnorm_relu_bwd"],
    "pk_wbce": ["wbce_kernel"],
    "pk_l2_normalize_fwd": ["l2norm_fwd_kernel"],
    "pk_l2_normalize_bwd": ["l2norm_bwd_kernel"],
}
# families whose launches are ONE of several kernels (every dispatch is a family launch)
ANY_LEAD = {"pk_linear_fwd+ex"}
# entry point -> its kernels, normalised per entry call with the bench's call count
PER_ENTRY = {"pk_linear_ex": FAMILIES["pk_linear_fwd+ex"],
             "pk_feat_dist_topk": FAMILIES["pk_feat_dist_topk"],
             "pk_linear_wgrad_grouped": FAMILIES["pk_linear_wgrad_grouped"],
             "pk_attention_fwd": FAMILIES["pk_attention_fwd"], "pk_attention_bwd": FAMILIES["pk_attention_bwd"]}
# (the first kernel of each family is counted once per family launch)


# the last kernel of every eager training step (pk_clip_rmsprop): dispatches after the last one
# belong to bench.py's roofline probes (the configs[3] ball-query probe, the feature-distance
# probe's 23 calls), not to a step
STEP_END = "clip_rmsprop_kernel"


def step_window_end(dirpath, counter):
    """Dispatch_Id of the last step's closing kernel (None: no such kernel, no window)."""
    end = None
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter and STEP_END in row["Kernel_Name"]:
                    d = int(row["Dispatch_Id"])
                    end = d if end is None else max(end, d)
    return end


def read(dirpath, counter, min_grid=0, max_grid=None, in_steps=True):
    """kernel name -> (dispatches, summed counter value), dispatches filtered by grid size and (in_steps)
    to the eager steps' window (Dispatch_Id up to the last step's closing kernel)."""
    tot = defaultdict(lambda: [0, 0.0])
    end = step_window_end(dirpath, counter) if in_steps else None
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                if end is not None and int(row["Dispatch_Id"]) > end:
                    continue
                grid = int(float(row.get("Grid_Size", 0) or 0))
                if grid < min_grid or (max_grid is not None and grid > max_grid):
                    continue
                t = tot[row["Kernel_Name"]]
                t[0] += 1
                t[1] += float(row["Counter_Value"])
    return tot


# bench.py's configs[3]-size ball-query probe (256 x 2048 x 2048) runs the mask kernel on a
# grid of 32 x 256 workgroups of 256 threads; the in-step launches are far smaller
PROBE_GRID = 32 * 256 * 256


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    res = {}
    for fam, names, lo, hi in [(f, n, 0, PROBE_GRID - 1) for f, n in FAMILIES.items()] + \
            [("pk_ball_query_mask@configs3_probe", FAMILIES["pk_ball_query_mask"], PROBE_GRID, None)]:
        steps = not fam.endswith("_probe")  # the probe entry: the dispatches after the steps
        fetch = read(fetch_dir, "FETCH_SIZE", lo, hi, in_steps=steps)
        write = read(write_dir, "WRITE_SIZE", lo, hi, in_steps=steps)
        def summed(tab, names=names, fam=fam):
            lead = names if fam in ANY_LEAD else names[:1]
            n_lead = sum(c for k, (c, _) in tab.items() if any(nm in k for nm in lead))
            v = sum(s for k, (_, s) in tab.items() if any(nm in k for nm in names))
            return n_lead, v
        nf, fb = summed(fetch)
        nw, wb = summed(write)
        if nf == 0 or nw == 0:
            continue
        fetch_b = 2.0 * fb * 1024 / nf   # KiB -> B, gfx950 x2 read correction, per launch
        write_b = wb * 1024 / nw
        res[fam] = {"fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
                    "traffic_bytes_per_launch": fetch_b + write_b, "launches": nf}
    if len(sys.argv) > 4:
        bench = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
        calls = {k: v["launches"] for k, v in bench.get("kernels", {}).items()}
        for ent, names in PER_ENTRY.items():
            n = calls.get(ent)
            if not n:
                continue
            fb = sum(s for k, (_, s) in read(fetch_dir, "FETCH_SIZE", 0, PROBE_GRID - 1).items()
                     if any(nm in k for nm in names))
            wb = sum(s for k, (_, s) in read(write_dir, "WRITE_SIZE", 0, PROBE_GRID - 1).items()
                     if any(nm in k for nm in names))
            fetch_b, write_b = 2.0 * fb * 1024 / n, wb * 1024 / n
            res[ent] = {"fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
                        "traffic_bytes_per_launch": fetch_b + write_b, "launches": n,
                        "per": "entry-point call (bench probe count)"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
