// Big-tile ping-pong MFMA GEMM for MI355X (gfx950): bf16 operands, fp32
// accumulate, C[M][N] = epilogue(A[M][K] * B[N][K]^T) -- the dense-operand
// contract of cgemm (kADense only), for the shapes where a workgroup can own a
// 256-row tile: BERT's projections at M = 128 x batch, ResNet's wide 1x1 convs.
//
// Why (round-5 VERDICT item 1, docs/benchmarks.md "Why the 32x32 builds did not
// halve the LDS traffic"): the cgemm tiles put 32 x 32 .. 64 x 96 outputs on a
// wave, below the m n / (m + n) >= 32 LDS-bytes-per-FLOP threshold, and every
// wave of a workgroup reads its fragments, waits and computes in lockstep, so
// the matrix pipe idles during every read burst (MFMA busy 10-22 %).  Here:
//
//   * 8 waves (2 along M x 4 along N), 128 x 64 / 48 / 32 outputs per wave
//     (256 x 256 / 192 / 128 tiles): accumulators 128 / 96 / 64 VGPRs per lane;
//   * each 64-deep K-tile runs as 4 phases, one 32-row part of the wave tile
//     each (all its columns: 16 / 12 / 8 v_mfma_f32_16x16x32_bf16 per wave);
//     the wave's B fragments are read once per K-tile, its A fragments in
//     phases 0-1 (so A's buffer frees early, BG::EARLY_A) or, for the
//     256 x 256 tile whose accumulators leave no room, half in phase 0 and
//     half in phase 2;
//   * ping-pong: a phase is [LOAD: issue its fragment reads and DMAs]
//     s_barrier [COMPUTE: wait for the reads, 16 MFMAs] s_barrier, and waves
//     4-7 (the second M half) start one barrier late, so on every SIMD one
//     wave computes while its partner loads: the matrix pipe is fed every
//     interval (cdna_hip_programming.md, 256^2 8-phase template and
//     MI355X_MICROARCH.md 'Two waves per SIMD' item 9);
//   * operands go HBM/L2 -> LDS by buffer_load ... lds (16 B per lane, 1-KB
//     pieces of 8 rows x 128 B), two K-tile buffers, refilled as soon as the
//     last phase that reads them is two phases back: B of tile u+2 in phase
//     (u,2), A of tile u+2 in (u,3) (EARLY_A) -- five phases of lead -- or A
//     of tile u+1 in (u,0) (three).  The only wait is one counted vmcnt per
//     K-tile, in phase (u,3), which leaves the next-but-one tile in flight;
//   * RAW / WAR by construction: a half is read one phase after the phase
//     whose LOAD segment waited for it (both groups have then passed a barrier
//     behind their waits) and refilled two phases after its last read (both
//     groups' lgkmcnt waits and a barrier lie between) -- the staggered-group
//     rules of cdna_hip_programming.md ("Read a staged buffer one phase
//     AFTER ...", "restage >= 2 phases after its last ds_read");
//   * LDS rows of 128 B with 16-B chunks XOR-swizzled by (row & 7), applied on
//     the DMA source address (the DMA image is lane-linear) and undone in the
//     fragment reads (conflict-free ds_read_b128, as cgemm);
//   * raw s_barrier only (a __syncthreads() would drain vmcnt, i.e. every DMA
//     in flight), all LDS in the one dynamic array;
//   * epilogue: bias + activation in registers and a bf16 tile staged once in
//     LDS (135 KB), then 16-B row stores; residual / fp32 / second-output /
//     split-K launches stage fp32 in two 128-row passes (each staged by the
//     group that owns those rows) and run the shared epi_chunk.
#include <algorithm>
#include <type_traits>

#include "gemm_common.h"
#include "cgemm.h"

namespace tfsk {

namespace {

using namespace gemm;

template <int BM, int BN>
struct BG {
  static constexpr int NW = 8, NT = 512;
  static constexpr int WGN = 4;                     // waves along N (2 along M: the ping-pong groups)
  static constexpr int WM = BM / 2, WN = BN / WGN;  // wave tile
  static constexpr int PART = WM / 4;               // rows per phase (4 phases per K-tile)
  static constexpr int PTM = PART / 16, TN = WN / 16;
  static constexpr int A_B = BM * 128, B_B = BN * 128;   // bytes of one K-tile of A / B
  static constexpr int BUF = A_B + B_B;
  static constexpr int PAT = BM / 8 / NW;           // 1-KB DMA pieces per wave per K-tile of A
  static constexpr int PBT = BN / 8 / NW;           // ... of B
  // Early A: every A fragment of a K-tile is read in its phases 0-1 (4 row
  // parts x 2 k-halves in registers), so A's buffer is free two phases
  // later and the next-but-one K-tile's A goes out in phase 3: five phases
  // of lead for both operands.  The 256 x 256 tile cannot hold all of A next
  // to its 128 accumulators; it reads parts 0-1 in phase 0 and 2-3 in phase 2
  // (A issued a K-tile ahead in phase 0: three phases of lead).
  static constexpr bool EARLY_A = BN <= 192;
  static constexpr int A_REG_PARTS = EARLY_A ? 4 : 2;
  static constexpr int CB_LD = BN + 8;              // bf16 staging row (elements)
  static constexpr int CS_LD = BN + 4;              // fp32 staging row (one 128-row pass)
  static constexpr int LDS_BF = BM * CB_LD * 2;
  static constexpr int LDS_F32 = (BM / 2) * CS_LD * 4;
  static constexpr int LDS = std::max(std::max(2 * BUF, LDS_BF), LDS_F32);
  static_assert(BM == 256 && (BN == 256 || BN == 192 || BN == 128), "tiles built: 256 x {256, 192, 128}");
  static_assert(PAT * 8 * NW == BM && PBT * 8 * NW == BN && PTM >= 1 && TN >= 1 && WN % 16 == 0, "tile split");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

template <int BM, int BN>
__global__ __launch_bounds__(512, 1) void bgemm_kernel(IGemmArgs p) {
  using G = BG<BM, BN>;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  char* const smem = reinterpret_cast<char*>(smem_raw);
  typedef __attribute__((address_space(3))) void* lds_ptr_t;

  // ---- tile of this workgroup (XCD remap + GROUP_M ordering, as cgemm)
  const int M = p.M, N = p.N;
  const int nbm = (M + BM - 1) / BM, nbn = (N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int kGroupM = 8;
  const int per_group = kGroupM * nbn;
  const int first_m = (wg / per_group) * kGroupM;
  const int gsz = min(nbm - first_m, kGroupM);
  const int bm = first_m + (wg % per_group) % gsz;
  const int bn = (wg % per_group) / gsz;
  const int m0 = bm * BM, n0 = bn * BN;
  trace_stamp(p, 0);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / G::WGN, wc = wid % G::WGN;   // wr = ping-pong group

  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.a), 0, int(p.a_bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.b), 0, int(p.b_bytes), 0x00020000);

  // ---- per-lane DMA source offsets: lane -> row lane>>3 of its 8-row piece,
  // LDS slot lane&7 holding logical chunk (lane&7) ^ (row & 7); wave w owns
  // the contiguous pieces w * PAT .. (A) and w * PBT .. (B)
  const uint32_t kc = uint32_t(((lane & 7) ^ (lane >> 3)) * 8);
  uint32_t a_off[G::PAT], b_off[G::PBT];
#pragma unroll
  for (int i = 0; i < G::PAT; ++i) {
    const int m = m0 + (wid * G::PAT + i) * 8 + (lane >> 3);
    a_off[i] = m < M ? (uint32_t(m) * uint32_t(p.lda) + kc) * 2u : kOOB;
  }
#pragma unroll
  for (int i = 0; i < G::PBT; ++i) {
    const int n = n0 + (wid * G::PBT + i) * 8 + (lane >> 3);
    b_off[i] = n < N ? (uint32_t(n) * uint32_t(p.ldb) + kc) * 2u : kOOB;
  }
  // k-tile range (split-K: blockIdx.y selects a slice)
  const int nk_all = p.K / KT;
  int kt0 = 0, nk = nk_all;
  if (p.splits > 1) {
    kt0 = blockIdx.y * p.kt_per_split;
    nk = min(nk_all - kt0, p.kt_per_split);
  }
  auto issue_a = [&](int t, int buf) {
    const uint32_t soff = uint32_t((kt0 + t) * KT) * 2u;
#pragma unroll
    for (int i = 0; i < G::PAT; ++i) {
      const uint32_t v = a_off[i];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_ptr_t)(smem + buf * G::BUF + (wid * G::PAT + i) * 1024),
                                               16, v, soff, 0, 0);
    }
  };
  auto issue_b = [&](int t, int buf) {
    const uint32_t soff = uint32_t((kt0 + t) * KT) * 2u;
#pragma unroll
    for (int i = 0; i < G::PBT; ++i) {
      const uint32_t v = b_off[i];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (lds_ptr_t)(smem + buf * G::BUF + G::A_B + (wid * G::PBT + i) * 1024), 16, v, soff, 0, 0);
    }
  };

  // ---- fragment read offsets (16x16x32: lane holds row l & 15, k chunk (l >> 4) + 4 kk)
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t sw0 = uint32_t((fq ^ (fr & 7)) << 4), sw1 = uint32_t(((4 + fq) ^ (fr & 7)) << 4);
  const uint32_t ra = uint32_t((wr * G::WM + fr) * 128);
  const uint32_t rb = uint32_t(G::A_B + (wc * G::WN + fr) * 128);

  f32x4 acc[4][G::PTM][G::TN];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < G::PTM; ++i)
#pragma unroll
      for (int j = 0; j < G::TN; ++j) acc[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[G::A_REG_PARTS][2][G::PTM], fb[2][G::TN];

  // A fragments of row parts q0 .. q0 + n - 1 into register slots s0 ..
  auto read_a = [&](int buf, int q0, int n, int s0) {
#pragma unroll
    for (int q = 0; q < n; ++q)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < G::PTM; ++i)
          fa[s0 + q][kk][i] = *reinterpret_cast<const bf16x8*>(smem + buf * G::BUF + ra + (q0 + q) * G::PART * 128 +
                                                               i * 16 * 128 + (kk ? sw1 : sw0));
  };
  auto read_b = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < G::TN; ++j)
        fb[kk][j] = *reinterpret_cast<const bf16x8*>(smem + buf * G::BUF + rb + j * 16 * 128 + (kk ? sw1 : sw0));
  };
  auto barrier = []() { __builtin_amdgcn_s_barrier(); };
  // COMPUTE segment of phase q: wait for this wave's reads, the row part's
  // MFMAs (register slot s of A), barrier
  auto compute = [&](auto qc, auto sc) {
    constexpr int q = decltype(qc)::value, sl = decltype(sc)::value;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < G::PTM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
          acc[q][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[sl][kk][i], fb[kk][j], acc[q][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    barrier();
  };
  auto load_end = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  // ---- prologue.  EARLY_A: tiles 0 and 1 whole, wait for tile 0.  Else:
  // tile 0 whole and tile 1's B, wait for tile 0 (tile 1's A goes out in
  // phase (0, 0)).
  if (nk > 0) {
    issue_a(0, 0);
    issue_b(0, 0);
    if (nk > 1) {
      if constexpr (G::EARLY_A) {
        issue_b(1, 1);
        issue_a(1, 1);
        wait_vmcnt<G::PAT + G::PBT>();
      } else {
        issue_b(1, 1);
        wait_vmcnt<G::PBT>();
      }
    } else {
      wait_vmcnt<0>();
    }
  }
  barrier();   // every wave's tile-0 DMAs landed (raw barrier: tile 1 stays in flight)
  trace_stamp(p, 1);
  if (wr == 1) barrier();   // the second group runs one barrier behind

  // ---- K loop: tiles in pairs, so the buffer index of every access is an immediate.
  // EARLY_A schedule of K-tile u (buffer b = u & 1):
  //   phase 0: read B, A parts 0-1      | part 0
  //   phase 1: read A parts 2-3         | part 1
  //   phase 2: B(u+2) -> b              | part 2   (B of u last read in phase 0)
  //   phase 3: A(u+2) -> b; wait u+1    | part 3   (A of u last read in phase 1)
  // late-A schedule (256 x 256):
  //   phase 0: read B, A parts 0-1; A(u+1) -> b^1   | part 0  (A of u-1 last read in its phase 2)
  //   phase 1: -                                    | part 1
  //   phase 2: read A parts 2-3; B(u+2) -> b        | part 2  (B of u last read in phase 0)
  //   phase 3: wait u+1                             | part 3
  auto tile = [&](auto bufc, int u) {
    constexpr int buf = decltype(bufc)::value;
    __builtin_amdgcn_sched_barrier(0);
    read_b(buf);
    read_a(buf, 0, 2, 0);
    if constexpr (!G::EARLY_A) {
      if (u + 1 < nk) issue_a(u + 1, buf ^ 1);
    }
    load_end();
    compute(I0{}, I0{});
    if constexpr (G::EARLY_A) read_a(buf, 2, 2, 2);
    load_end();
    compute(I1{}, I1{});
    if constexpr (!G::EARLY_A) read_a(buf, 2, 2, 0);
    if (u + 2 < nk) issue_b(u + 2, buf);
    load_end();
    if constexpr (G::EARLY_A) compute(I2{}, I2{});
    else compute(I2{}, I0{});
    if constexpr (G::EARLY_A) {
      if (u + 2 < nk) {
        issue_a(u + 2, buf);
        wait_vmcnt<G::PAT + G::PBT>();
      } else if (u + 1 < nk) {
        wait_vmcnt<0>();
      }
    } else {
      if (u + 2 < nk) wait_vmcnt<G::PBT>();
      else if (u + 1 < nk) wait_vmcnt<0>();
    }
    load_end();
    if constexpr (G::EARLY_A) compute(I3{}, I3{});
    else compute(I3{}, I1{});
  };
  for (int u = 0; u < nk; u += 2) {
    tile(std::integral_constant<int, 0>{}, u);
    if (u + 1 < nk) tile(std::integral_constant<int, 1>{}, u + 1);
  }
  if (wr == 0) barrier();   // re-join the groups
  wait_vmcnt<0>();
  __syncthreads();
  trace_stamp(p, 2);

  // ---- epilogue
  // C/D of 16x16x32: column lane & 15, rows 4 (lane >> 4) + r
  auto row_of = [&](int q, int i, int r) { return wr * G::WM + q * G::PART + i * 16 + fq * 4 + r; };
  auto col_of = [&](int j) { return wc * G::WN + j * 16 + fr; };
  if (p.splits <= 1 && p.residual == nullptr && p.out2 == nullptr && !p.out_f32 && p.out != nullptr &&
      p.act != kActGeluErf && !p.epi_f32) {
    uint16_t* Cb = reinterpret_cast<uint16_t*>(smem);
    const bool use_b = p.bias != nullptr && p.N % 8 == 0;
    const __amdgpu_buffer_rsrc_t rsb =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.bias), 0, use_b ? p.N * 4 : 0, 0x00020000);
    float bj[G::TN];
#pragma unroll
    for (int j = 0; j < G::TN; ++j)
      bj[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsb, uint32_t(n0 + col_of(j)) * 4u, 0, 0));
    const float alpha = p.alpha;
    auto stage = [&](auto actc) __attribute__((always_inline)) {
      constexpr int ACT = decltype(actc)::value;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < G::PTM; ++i)
#pragma unroll
          for (int j = 0; j < G::TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = act_fn<ACT>(acc[q][i][j][r] * alpha + bj[j] + 0.f);
              Cb[row_of(q, i, r) * G::CB_LD + col_of(j)] = __builtin_bit_cast(uint16_t, static_cast<__bf16>(v));
            }
    };
    switch (p.act) {
      case kActRelu: stage(std::integral_constant<int, kActRelu>{}); break;
      case kActGeluTanh: stage(std::integral_constant<int, kActGeluTanh>{}); break;
      case kActTanh: stage(std::integral_constant<int, kActTanh>{}); break;
      default: stage(std::integral_constant<int, kActNone>{}); break;
    }
    __syncthreads();
    constexpr int CPRB = BN / 8;
#pragma unroll 4
    for (int it = 0; it < BM * CPRB / G::NT; ++it) {
      const int c = tid + it * G::NT, row = c / CPRB, ch = c - row * CPRB;
      const int m = m0 + row, n = n0 + ch * 8;
      if (m < M && n < N)
        *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p.out) + size_t(m) * p.ldc + n) =
            *reinterpret_cast<const uint4*>(Cb + row * G::CB_LD + ch * 8);
    }
    trace_stamp(p, 3);
    return;
  }

  // fp32 image in two 128-row passes: pass ps holds the rows of group ps
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int RPP = BM / 2;
  using E = Epi<RPP, BN, G::NT>;
  float4 bias0, bias1;
  prefetch_bias<RPP, BN, G::NT>(p, n0, tid, bias0, bias1);
  const float bv[8] = {bias0.x, bias0.y, bias0.z, bias0.w, bias1.x, bias1.y, bias1.z, bias1.w};
#pragma unroll
  for (int ps = 0; ps < 2; ++ps) {
    if (ps > 0) __syncthreads();   // the previous pass has been read
    if (wr == ps) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < G::PTM; ++i)
#pragma unroll
          for (int j = 0; j < G::TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              Cs[(row_of(q, i, r) - ps * RPP) * G::CS_LD + col_of(j)] = acc[q][i][j][r];
    }
    __syncthreads();
    const int mp = m0 + ps * RPP;
    if (p.splits > 1) {
      // raw (alpha-scaled) partial slab of this K slice; splitk_reduce applies the epilogue
      const float alpha = p.alpha;
      float* ws = p.ws + size_t(blockIdx.y) * M * N;
      for (int it = 0; it < E::ITERS; ++it) {
        int row, col;
        if (!epi_rowcol<RPP, BN, G::NT>(tid, it, row, col)) continue;
        const int m = mp + row, n = n0 + col;
        if (m >= M || n >= N) continue;
        const float* src = Cs + row * G::CS_LD + col;
        float4 a = *reinterpret_cast<const float4*>(src);
        float4 b = *reinterpret_cast<const float4*>(src + 4);
        a.x *= alpha; a.y *= alpha; a.z *= alpha; a.w *= alpha;
        b.x *= alpha; b.y *= alpha; b.z *= alpha; b.w *= alpha;
        float* dst = ws + size_t(m) * N + n;
        *reinterpret_cast<float4*>(dst) = a;
        *reinterpret_cast<float4*>(dst + 4) = b;
      }
      continue;
    }
    auto run = [&](auto actc) {
      constexpr int ACT = decltype(actc)::value;
#pragma unroll 2
      for (int it = 0; it < E::ITERS; ++it) {
        int row, col;
        if (!epi_rowcol<RPP, BN, G::NT>(tid, it, row, col)) continue;
        const int m = mp + row, n = n0 + col;
        if (m >= M || n >= N) continue;
        const uint4 rr = p.residual ? *reinterpret_cast<const uint4*>(p.residual + size_t(m) * p.ldr + n)
                                    : make_uint4(0, 0, 0, 0);
        epi_chunk<ACT>(p, Cs + row * G::CS_LD + col, m, n, bv, rr);
      }
    };
    switch (p.act) {
      case kActRelu: run(std::integral_constant<int, kActRelu>{}); break;
      case kActGeluTanh: run(std::integral_constant<int, kActGeluTanh>{}); break;
      case kActGeluErf: run(std::integral_constant<int, kActGeluErf>{}); break;
      case kActTanh: run(std::integral_constant<int, kActTanh>{}); break;
      default: run(std::integral_constant<int, kActNone>{}); break;
    }
  }
  trace_stamp(p, 3);
}

template <int BM, int BN>
hipError_t launch_bg(const IGemmArgs& a0, hipStream_t s) {
  using G = BG<BM, BN>;
  IGemmArgs a = a0;
  a.epi_f32 = epi_f32_env();
  const int nk = a.K / KT;
  const int splits = a.splits > 1 ? a.splits : 1;
  if (splits > 1) a.kt_per_split = (nk + splits - 1) / splits;
  const long tiles = long((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (tiles == 0) return hipSuccess;
  if (tiles >= (1L << 31)) return hipErrorInvalidValue;
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&bgemm_kernel<BM, BN>), G::LDS);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((bgemm_kernel<BM, BN>), dim3(unsigned(tiles), splits), dim3(G::NT), G::LDS, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t bgemm_launch(const IGemmArgs& a, int a_mode, int idx, hipStream_t s) {
  if (a_mode != kADense) return hipErrorInvalidValue;     // dense operands only
  if (a.counters != nullptr) return hipErrorInvalidValue; // no in-kernel split-K fixup
  if (a.st_out != nullptr || a.a_st != nullptr || a.r_st != nullptr) return hipErrorInvalidValue;   // no deferred LN
  switch (idx) {
    case 0: return launch_bg<256, 256>(a, s);
    case 1: return launch_bg<256, 128>(a, s);
    case 2: return launch_bg<256, 192>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tfsk
