// FETCH_SIZE / WRITE_SIZE calibration on the replay kernel's own access widths.
//
// Each kernel touches a known number of bytes of a 1 GiB buffer (past the 256 MiB Infinity Cache), once;
// running this under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE` gives the counter
// value per dispatch against that byte count.  Patterns (mtb_replay.hip):
//   rd_dword      64 lanes x 4 B contiguous per wave-instruction (a 320-B block record's 256-B body)
//   rd_rec320     one 320-B record per wave: 64 x 4 B + 5 x 4 B of its header (load_view / stage_rec)
//   rd_went16     64 lanes x 16 B (window-list entries, WEnt)
//   rd_scatter4   one lane, 4 B, in a distinct 128-B line per access (segp / aux / heap reads)
//   wr_dword      64 lanes x 4 B contiguous stores (record write-back, place_children)
//   wr_scatter4   one lane, 4 B stores, a distinct 128-B line each (set_meta / add_len_levels / counts)
// Prints one line per kernel: name, algorithmic bytes.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHK(x)                                                                              \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                               \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

static constexpr uint64_t BUF = 1ull << 30;  // bytes
static constexpr int WAVES = 256 * 16;       // grid of 64-lane workgroups

__global__ void __launch_bounds__(64) rd_dword(const uint32_t* __restrict__ p, uint64_t words, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 64) acc += p[i];
  if (acc == 0x9E3779B9u) sink[0] = acc;
}
__global__ void __launch_bounds__(64) rd_rec320(const uint32_t* __restrict__ p, uint64_t recs, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t r = blockIdx.x; r < recs; r += gridDim.x) {
    const uint32_t* q = p + r * 80;
    acc += q[threadIdx.x];
    if (threadIdx.x < 5) acc += q[64 + threadIdx.x];
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}
__global__ void __launch_bounds__(64) rd_went16(const uint4* __restrict__ p, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 64) {
    const uint4 v = p[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}
__global__ void __launch_bounds__(64) rd_scatter4(const uint32_t* __restrict__ p, uint64_t lines, uint32_t* sink) {
  uint32_t acc = 0;
  if (threadIdx.x == 0)
    for (uint64_t l = blockIdx.x; l < lines; l += gridDim.x) acc += p[l * 32];
  if (acc == 0x9E3779B9u) sink[0] = acc;
}
__global__ void __launch_bounds__(64) wr_dword(uint32_t* __restrict__ p, uint64_t words) {
  for (uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 64) p[i] = (uint32_t)i;
}
__global__ void __launch_bounds__(64) wr_scatter4(uint32_t* __restrict__ p, uint64_t lines) {
  if (threadIdx.x == 0)
    for (uint64_t l = blockIdx.x; l < lines; l += gridDim.x) p[l * 32] = (uint32_t)l;
}

int main() {
  uint32_t *buf, *sink;
  CHK(hipMalloc(&buf, BUF));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(buf, 1, BUF));
  const uint64_t words = BUF / 4, recs = BUF / 320, lines = BUF / 128;
  // each pattern runs on a buffer it has not touched since the last flush-sized sweep (1 GiB > L2 + L3)
  hipLaunchKernelGGL(rd_dword, dim3(WAVES), dim3(64), 0, 0, buf, words, sink);
  CHK(hipDeviceSynchronize());
  printf("rd_dword %llu\n", (unsigned long long)(words * 4));
  hipLaunchKernelGGL(rd_rec320, dim3(WAVES), dim3(64), 0, 0, buf, recs, sink);
  CHK(hipDeviceSynchronize());
  printf("rd_rec320 %llu\n", (unsigned long long)(recs * 276));
  hipLaunchKernelGGL(rd_went16, dim3(WAVES), dim3(64), 0, 0, reinterpret_cast<const uint4*>(buf), BUF / 16, sink);
  CHK(hipDeviceSynchronize());
  printf("rd_went16 %llu\n", (unsigned long long)BUF);
  hipLaunchKernelGGL(rd_scatter4, dim3(WAVES), dim3(64), 0, 0, buf, lines, sink);
  CHK(hipDeviceSynchronize());
  printf("rd_scatter4 %llu (lines %llu)\n", (unsigned long long)(lines * 4), (unsigned long long)lines);
  hipLaunchKernelGGL(wr_dword, dim3(WAVES), dim3(64), 0, 0, buf, words);
  CHK(hipDeviceSynchronize());
  printf("wr_dword %llu\n", (unsigned long long)(words * 4));
  hipLaunchKernelGGL(wr_scatter4, dim3(WAVES), dim3(64), 0, 0, buf, lines);
  CHK(hipDeviceSynchronize());
  printf("wr_scatter4 %llu (lines %llu)\n", (unsigned long long)(lines * 4), (unsigned long long)lines);
  CHK(hipFree(buf));
  CHK(hipFree(sink));
  return 0;
}
