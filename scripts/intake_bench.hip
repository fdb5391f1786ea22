// Per-CU operand intake micro-benchmark (MI355X / gfx950).
//
// How many bytes per second can ONE CU pull from an L2-resident buffer, by
// load form and waves per workgroup?  This bounds every tiled GEMM here: a
// BM x BN tile needs (BM + BN) * 128 B per 64-deep k-step for BM*BN*64 MACs.
//
//   mode 0: global_load_dwordx4 into VGPRs (xor-reduced so nothing is dropped)
//   mode 1: buffer_load_dword ... lds, 16 B per lane (LDS-DMA), counted vmcnt
//
// Every workgroup sweeps the same `span`-byte window (L2 / Infinity-Cache
// resident after the first pass) `reps` times; one workgroup per CU.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/intake_bench scripts/intake_bench.hip
//   /tmp/intake_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int NT, int DEPTH>
__global__ __launch_bounds__(NT) void regs_kernel(const uint4* __restrict__ src, size_t span16, int reps,
                                                  unsigned* __restrict__ sink) {
  const int tid = threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  // each WG starts at a different offset so the WGs do not march in lockstep
  const size_t start = (size_t(blockIdx.x) * 4096) % span16;
  for (int r = 0; r < reps; ++r) {
    for (size_t i = tid; i < span16; i += size_t(NT) * DEPTH) {
      uint4 v[DEPTH];
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        size_t j = i + size_t(d) * NT;
        j = j < span16 ? j : i;
        j += start;
        if (j >= span16) j -= span16;
        v[d] = src[j];
      }
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        acc.x ^= v[d].x; acc.y ^= v[d].y; acc.z ^= v[d].z; acc.w ^= v[d].w;
      }
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[tid] = acc.x;   // practically never: keeps the loads
}

template <int NT, int SLOTS>
__global__ __launch_bounds__(NT) void lds_kernel(const char* __restrict__ src, int span, int reps,
                                                 unsigned* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src), 0, span, 0x00020000);
  const int tid = threadIdx.x, wid = tid >> 6;
  constexpr int NW = NT / 64;
  constexpr int SLOT_B = NT * 16;                   // bytes per issue round (1 KiB per wave)
  const int per_round = SLOT_B;
  const int rounds = span / per_round;
  const int start = int((size_t(blockIdx.x) * 4096) % size_t(span)) / per_round;
  int slot = 0;
  for (int r = 0; r < reps; ++r) {
    for (int k = 0; k < rounds; ++k) {
      int kk = k + start;
      if (kk >= rounds) kk -= rounds;
      const uint32_t voff = uint32_t(kk * per_round + tid * 16);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(smem + slot * SLOT_B + wid * 1024), 16, voff, 0, 0, 0);
      slot = slot + 1 == SLOTS ? 0 : slot + 1;
      __builtin_amdgcn_s_waitcnt((SLOTS - 1 & 15) | (((SLOTS - 1) >> 4) << 14) | (7 << 4) | (15 << 8));
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (reinterpret_cast<const unsigned*>(smem)[tid] == 0x12345678u) sink[tid] = 1;
  (void)NW;
}

template <typename F>
float time_it(F launch) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t spans[] = {size_t(2) << 20, size_t(16) << 20, size_t(64) << 20};
  unsigned* sink;
  CHECK(hipMalloc(&sink, 4096 * sizeof(unsigned)));
  for (size_t span : spans) {
  char* buf;
  CHECK(hipMalloc(&buf, span));
  CHECK(hipMemset(buf, 1, span));
  // a sweep per workgroup of a window larger than L2 comes from the Infinity Cache
  const int reps = span > (size_t(2) << 20) ? 1 : 8;
  const double bytes_per_wg = double(span) * reps;
  std::printf("CUs %d, window %zu KiB, %d sweeps per workgroup\n", cus, span >> 10, reps);
  auto report = [&](const char* what, int wgs, float ms) {
    const double per_cu = bytes_per_wg * wgs / cus / (ms * 1e-3) / 1e9;
    std::printf("%-40s wgs %4d  %8.3f ms  %7.1f GB/s per CU  %6.2f TB/s chip\n", what, wgs, ms, per_cu,
                per_cu * cus / 1e3);
  };
#define REGS(NT, D, WPC)                                                                                   \
  {                                                                                                        \
    const int wgs = cus * WPC;                                                                             \
    float ms = time_it([&] {                                                                               \
      hipLaunchKernelGGL((regs_kernel<NT, D>), dim3(wgs), dim3(NT), 0, 0, (const uint4*)buf, span / 16,     \
                         reps, sink);                                                                      \
    });                                                                                                    \
    report("regs nt=" #NT " depth=" #D " wg/cu=" #WPC, wgs, ms);                                           \
  }
  REGS(256, 4, 1) REGS(256, 8, 1) REGS(512, 4, 1) REGS(512, 8, 1) REGS(1024, 4, 1) REGS(1024, 8, 1)
  REGS(256, 8, 2) REGS(256, 8, 4)
#define LDS(NT, SL, WPC)                                                                                   \
  {                                                                                                        \
    const int wgs = cus * WPC;                                                                             \
    const int lds = NT * 16 * SL;                                                                          \
    float ms = time_it([&] {                                                                               \
      hipLaunchKernelGGL((lds_kernel<NT, SL>), dim3(wgs), dim3(NT), lds, 0, (const char*)buf, int(span),    \
                         reps, sink);                                                                      \
    });                                                                                                    \
    report("ldsdma nt=" #NT " inflight=" #SL " wg/cu=" #WPC, wgs, ms);                                     \
  }
  LDS(256, 4, 1) LDS(256, 8, 1) LDS(256, 16, 1) LDS(512, 8, 1) LDS(512, 16, 1) LDS(1024, 8, 1) LDS(256, 8, 2)
  CHECK(hipFree(buf));
  }
  CHECK(hipFree(sink));
  return 0;
}
