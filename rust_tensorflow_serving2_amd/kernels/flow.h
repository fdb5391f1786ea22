// Persistent dataflow executor for a chain of conv / GEMM layers (flow.hip).
//
// A small-batch ResNet forward is a chain of ~50 dependent convolutions whose
// kernels are each far too small to fill the chip: at batch 1 every launch
// pays the dependent-kernel boundary plus its own fill and drain, and the
// forward is a latency chain (profiles/round2/r50_b1_replay_stempool.txt:
// 58 dispatches of 4.7-11 us).  flow_kernel runs the whole chain as ONE
// launch: workgroups pull (layer, tile, K-slice) tasks from a device-wide
// ticket in program order, prefetch the task's weights into their LDS ring
// while the layer's producers are still running, wait on the producers'
// per-layer completion counters, and publish their own tile when done.
// Tickets are dealt in topological order, so a workgroup only ever waits on
// tasks already held by running workgroups: no deadlock whatever the residency.
#pragma once
#include <stdint.h>

#include "launch.h"

namespace tfsk {

// A pointer field of FlowStep: (kind << 60) | byte offset.  kind 0 = the
// per-call activation arena, 1 = the chain's input tensor, 2 = the chain's
// output tensor, 3 = an absolute device address (weights / bias).
constexpr int kFlowRefShift = 60;
constexpr int kFlowMaxSteps = 64;

// a_mode of a step (same operand forms as cgemm.hip)
enum FlowMode : int32_t { kFlowDense = 0, kFlowIm2col = 1, kFlowDual = 2 };

struct FlowStep {
  int64_t a, a2, w, bias, res, out, ws, pad64;
  int32_t M, N, K, K1, lda, ldb;
  int32_t H, W, C, Ho, Wo, KH, KW, SH, SW, PT, PL;
  int32_t mode, act, ntm, ntn, splits, ktps, ntasks;
  // producer steps (-1: none) of the operand a (its rows: the same rows for
  // dense / dual, the im2col window), a2 (dual: the strided 1x1 samples) and
  // the residual (same rows); split-K arrival counters (ctrl ints)
  int32_t dep_a, dep_a2, dep_res, ctr;
  int32_t a_bytes, a2_bytes, b_bytes;
  int32_t rctr;                          // this step's row-block counters: ctrl[rctr + bm * kFlowRowStride]
};
static_assert(sizeof(FlowStep) == 192, "FlowStep layout is mirrored by graph/flow.py");

// Table = int32 task0[kFlowMaxSteps] (first task id of each step, INT32_MAX
// past the last) followed by FlowStep[nsteps].  ctrl (ints, zero when first
// used): [0] ticket and [1] exit count (re-zeroed by the last workgroup out),
// [2] error flag (sticky: a dependency wait timed out), [3] epoch (launches
// completed), then the split-K arrival counters (re-zeroed by each tile's
// last slice) and the row-block counters.  A row-block counter counts the
// tiles of that 32-row block completed over ALL launches: launch e waits for
// (e + 1) * tiles-per-row (wrap-around compare), so nothing needs re-zeroing
// and a consumer tile waits only for the producer rows it reads.
constexpr int kFlowTileM = 32, kFlowTileN = 64;
constexpr int kFlowCtrlHead = 4;
constexpr int kFlowRowStride = 16;    // ints between row-block counters (one 64-B sector each)

hipError_t flow_launch(const void* table, int nsteps, int ntasks, void* arena, const void* entry, void* out,
                       int* ctrl, int grid, hipStream_t stream);

}  // namespace tfsk
