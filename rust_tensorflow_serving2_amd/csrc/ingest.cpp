// fp32 -> bf16 ingest conversion (see ingest.h).  AVX-512 BF16 when the CPU
// has it (one vcvtne2ps2bf16 per 32 values), scalar round-to-nearest-even
// otherwise.  Both give the same bits for every input, and the same bits as
// the device's v_cvt_pk_bf16_f32 under HIP's default fp32 mode (denormals
// kept): NaNs stay NaN and fp32 denormals round to bf16 denormals.
// vcvtne2ps2bf16 reads denormal inputs as zero, so a 32-value block holding
// one goes through the scalar path (one mask test per block otherwise).
#include "ingest.h"

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>

namespace tfs {

namespace {

inline uint16_t bf16_rne(uint32_t u) {
  if ((u & 0x7fffffffu) > 0x7f800000u) return uint16_t((u >> 16) | 0x40u);   // quiet NaN
  return uint16_t((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

void convert_scalar(uint16_t* dst, const uint8_t* src, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    uint32_t u;
    std::memcpy(&u, src + 4 * i, 4);
    dst[i] = bf16_rne(u);
  }
}

// Rows of at least kNtMin values are written with non-temporal 64-B stores:
// the pinned batch row is read next by the GPU's copy engine, never by this
// core, so the read-for-ownership a normal store pays on each line is wasted
// memory traffic (TFSERVE_INGEST_NT=0: plain stores).
constexpr size_t kNtMin = 4096;
const bool g_nt = [] {
  const char* e = getenv("TFSERVE_INGEST_NT");
  return !(e && std::atoi(e) == 0);
}();

__attribute__((target("avx512f,avx512bf16,avx512vl")))
void convert_avx512(uint16_t* dst, const uint8_t* src, size_t n) {
  size_t i = 0;
  const bool nt = g_nt && n >= kNtMin;
  if (nt) {
    // head: up to the first 64-B aligned output address
    const size_t mis = (reinterpret_cast<uintptr_t>(dst) & 63) / 2;
    const size_t head = (reinterpret_cast<uintptr_t>(dst) & 1) ? n : (mis ? 32 - mis : 0);
    if (head >= n) {
      convert_scalar(dst, src, n);
      return;
    }
    if (head) convert_scalar(dst, src, head);
    i = head;
    const __m512i ex = _mm512_set1_epi32(0x7f800000), mt = _mm512_set1_epi32(0x007fffff);
    for (; i + 32 <= n; i += 32) {
      const __m512 a = _mm512_loadu_ps(reinterpret_cast<const float*>(src + 4 * i));
      const __m512 b = _mm512_loadu_ps(reinterpret_cast<const float*>(src + 4 * i + 64));
      const __m512i ia = _mm512_castps_si512(a), ib = _mm512_castps_si512(b);
      const __mmask16 da = _mm512_mask_test_epi32_mask(_mm512_testn_epi32_mask(ia, ex), ia, mt);
      const __mmask16 db = _mm512_mask_test_epi32_mask(_mm512_testn_epi32_mask(ib, ex), ib, mt);
      if (__builtin_expect((da | db) != 0, 0)) {
        convert_scalar(dst + i, src + 4 * i, 32);
        continue;
      }
      const __m512bh r = _mm512_cvtne2ps_pbh(b, a);
      _mm512_stream_si512(reinterpret_cast<__m512i*>(dst + i), reinterpret_cast<__m512i>(r));
    }
    if (i < n) convert_scalar(dst + i, src + 4 * i, n - i);
    _mm_sfence();   // the row is handed to another thread / the copy engine next
    return;
  }
  for (; i + 32 <= n; i += 32) {
    const __m512 a = _mm512_loadu_ps(reinterpret_cast<const float*>(src + 4 * i));
    const __m512 b = _mm512_loadu_ps(reinterpret_cast<const float*>(src + 4 * i + 64));
    // denormal lanes: exponent 0, mantissa != 0
    const __m512i ex = _mm512_set1_epi32(0x7f800000), mt = _mm512_set1_epi32(0x007fffff);
    const __m512i ia = _mm512_castps_si512(a), ib = _mm512_castps_si512(b);
    const __mmask16 da = _mm512_mask_test_epi32_mask(_mm512_testn_epi32_mask(ia, ex), ia, mt);
    const __mmask16 db = _mm512_mask_test_epi32_mask(_mm512_testn_epi32_mask(ib, ex), ib, mt);
    if (__builtin_expect((da | db) != 0, 0)) {
      convert_scalar(dst + i, src + 4 * i, 32);
      continue;
    }
    // (b, a): the low 16 lanes of the result come from the second operand
    const __m512bh r = _mm512_cvtne2ps_pbh(b, a);
    _mm512_storeu_si512(reinterpret_cast<void*>(dst + i), reinterpret_cast<__m512i>(r));
  }
  if (i < n) convert_scalar(dst + i, src + 4 * i, n - i);
}

using ConvFn = void (*)(uint16_t*, const uint8_t*, size_t);

ConvFn pick() {
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512bf16") && __builtin_cpu_supports("avx512vl")) return convert_avx512;
  return convert_scalar;
}

const ConvFn g_conv = pick();

}  // namespace

void ingest_f32_to_bf16(uint16_t* dst, const uint8_t* src, size_t n) {
  if (n) g_conv(dst, src, n);
}

void ingest_rows(uint8_t* dst, const uint8_t* src, size_t wire_bytes, int conv) {
  if (conv == 1) {
    ingest_f32_to_bf16(reinterpret_cast<uint16_t*>(dst), src, wire_bytes / 4);
  } else {
    std::memcpy(dst, src, wire_bytes);
  }
}

}  // namespace tfs
