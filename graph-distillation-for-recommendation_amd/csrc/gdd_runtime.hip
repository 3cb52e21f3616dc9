// gdd_runtime.hip — error state, ABI version, device check, and the hipcub-backed scan/sort
// primitives the kernels share.
#include "gdd_common.hpp"

#include <hipcub/hipcub.hpp>

namespace gdd {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

size_t scan_i32_ws_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                   (int)n);
  return align256(bytes);
}

int exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t ws_bytes,
                       hipStream_t s) {
  size_t need = 0;
  GDD_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, need, in, out, (int)n, s));
  if (need > ws_bytes) return fail(GDD_E_WORKSPACE, "scan workspace %zu < %zu", ws_bytes, need);
  GDD_HIP(hipcub::DeviceScan::ExclusiveSum(ws, need, in, out, (int)n, s));
  return GDD_OK;
}

size_t sort_pairs_ws_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
  return align256(bytes);
}

// stable LSD radix sort of (key, value) pairs on bits [0, end_bit)
int sort_pairs_i32(const int32_t* keys_in, int32_t* keys_out, const int32_t* vals_in,
                   int32_t* vals_out, int64_t n, int end_bit, void* ws, size_t ws_bytes,
                   hipStream_t s) {
  size_t need = 0;
  GDD_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, need, keys_in, keys_out, vals_in, vals_out,
                                             (int)n, 0, end_bit, s));
  if (need > ws_bytes) return fail(GDD_E_WORKSPACE, "sort workspace %zu < %zu", ws_bytes, need);
  GDD_HIP(hipcub::DeviceRadixSort::SortPairs(ws, need, keys_in, keys_out, vals_in, vals_out,
                                             (int)n, 0, end_bit, s));
  return GDD_OK;
}

// streaming copy used to measure the achievable HBM bandwidth on the box (report the
// measured copy peak beside the 8 TB/s spec). Grid-stride over 16-byte words, 4 in flight per lane,
// nontemporal: the fastest of the shapes tools/probe/copy_probe.hip compares (~6.1 TB/s on 1 GiB).
typedef float v4f __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream_copy(const v4f* __restrict__ src,
                                                     v4f* __restrict__ dst, int64_t n16) {
  const int64_t step = (int64_t)gridDim.x * 1024;
  for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += step) {
    v4f v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = i + u * 256;
      if (j < n16) v[u] = __builtin_nontemporal_load(src + j);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = i + u * 256;
      if (j < n16) __builtin_nontemporal_store(v[u], dst + j);
    }
  }
}

}  // namespace gdd

extern "C" {

int gdd_stream_copy(const void* src, void* dst, size_t bytes, gdd_stream_t stream) {
  GDD_REQUIRE(src && dst && bytes % 16 == 0, "stream_copy: 16-byte multiple and non-null buffers");
  GDD_REQUIRE(((uintptr_t)src | (uintptr_t)dst) % 16 == 0, "stream_copy: 16-byte aligned buffers");
  const int64_t n16 = (int64_t)(bytes / 16);
  if (n16 == 0) return GDD_OK;
  const int64_t want = (n16 + 1023) / 1024;
  const unsigned g = (unsigned)(want < 8192 ? want : 8192);
  gdd::k_stream_copy<<<g, 256, 0, gdd::to_hip(stream)>>>(static_cast<const gdd::v4f*>(src),
                                                        static_cast<gdd::v4f*>(dst), n16);
  GDD_LAUNCHED();
  return GDD_OK;
}

const char* gdd_last_error(void) { return gdd::g_last_error.c_str(); }

int gdd_abi_version(void) { return 1; }

int gdd_device_ok(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  return std::string(prop.gcnArchName).rfind("gfx950", 0) == 0 ? 1 : 0;
}

}  // extern "C"
