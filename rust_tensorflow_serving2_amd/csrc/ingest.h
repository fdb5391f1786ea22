// Request ingest conversion: fp32 tensor payload -> bf16 batch rows.
//
// A servable whose first device op reads its fp32 input as bf16 anyway (the
// ResNet stem rounds every pixel to bf16 before its MFMAs) takes that input
// as bf16 rows: the IO threads convert while they copy a request into its
// pinned batch row, so the row, the host->device copy and the kernel's read
// are half the bytes of the fp32 wire tensor.  Rounding is round-to-nearest-
// even, the same as the device conversion (v_cvt_pk_bf16_f32, fp32
// denormals kept as bf16 denormals), so the results are bit-identical to
// feeding fp32 (tests/test_ingest.py pins the host bits, including
// denormals; tests/test_resnet_gpu.py the device parity).
#pragma once
#include <cstddef>
#include <cstdint>

namespace tfs {

// dst[i] = bf16(src float i), i < n; src may be unaligned (wire bytes).
void ingest_f32_to_bf16(uint16_t* dst, const uint8_t* src, size_t n);

// Copy `wire_bytes` of a tensor payload into a row: raw (conv 0) or fp32 ->
// bf16 (conv 1, the row receives wire_bytes / 2 bytes).
void ingest_rows(uint8_t* dst, const uint8_t* src, size_t wire_bytes, int conv);

}  // namespace tfs
