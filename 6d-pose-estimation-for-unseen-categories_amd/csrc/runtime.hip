// Runtime helpers of the pipelined executors (host code, no kernels).
//
// pk_stream_create_cu_mask: a HIP stream whose kernels run only on the CUs of `mask` (bit i of
// word i / 32 = CU i; hipExtStreamCreateWithCUMask). PipelinedTrainer / PipelinedInfer give the
// crop-formation stream a few CUs and the training stream the complement, so the latency-bound
// one-workgroup-per-crop kernels (FPS, SOR) do not share CUs with the wide training kernels
// (whose last round of blocks otherwise waits on the CUs the crop kernels hold).
#include "common.hpp"

extern "C" int pk_device_cu_count(int* out) {
  PK_REQUIRE(out != nullptr);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(out, hipDeviceAttributeMultiprocessorCount, dev);
  return e == hipSuccess ? PK_OK : (int)e;
}

extern "C" int pk_stream_create_cu_mask(const uint32_t* mask, int words, void** stream) {
  PK_REQUIRE(mask != nullptr && words > 0 && stream != nullptr);
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (e != hipSuccess) return (int)e;
  *stream = s;
  return PK_OK;
}

extern "C" int pk_stream_get_cu_mask(void* stream, int words, uint32_t* mask) {
  PK_REQUIRE(stream != nullptr && mask != nullptr && words > 0);
  const hipError_t e = hipExtStreamGetCUMask(static_cast<hipStream_t>(stream), (uint32_t)words, mask);
  return e == hipSuccess ? PK_OK : (int)e;
}

extern "C" int pk_stream_destroy(void* stream) {
  PK_REQUIRE(stream != nullptr);
  const hipError_t e = hipStreamDestroy(static_cast<hipStream_t>(stream));
  return e == hipSuccess ? PK_OK : (int)e;
}

// pk_build_id: the sha256 the Makefile formed over the sources this library was built from
// (build/build_id.c, regenerated whenever a source, the header or the Makefile changes).
extern "C" const char pk_build_id_str[];

extern "C" int pk_build_id(char* out, int cap) {
  PK_REQUIRE(out != nullptr && cap >= 65);
  for (int i = 0; i < 65; ++i) out[i] = pk_build_id_str[i];
  return PK_OK;
}
