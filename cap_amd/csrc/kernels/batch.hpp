// batch.hpp -- batch-level helper kernels (batch.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../../include/jg.h"
#include "common.hpp"

void launch_scatter(const int32_t* perm, const uint8_t* verdict_pad, uint8_t* verdict, int64_t npad, hipStream_t s);

// Device half of a pipeline chunk's dispatch plan.  The host counts jobs per
// bucket (kernel class x key; the reject bucket last) and sends the bucket
// cursors and padding ranges; this kernel places every caller job into the
// padded (class, key)-sorted order as a 16-byte JobDev and writes perm.
struct PlanFillArgs {
  const jg_tok* toks;               // the chunk's jobs in caller order
  int64_t n;
  uint64_t base;                    // arena offset of the chunk's device copy
  const uint8_t* cls_tab;           // [key * 16 + alg] -> kernel class (0 = reject)
  int32_t nkeys;
  unsigned long long* cursor;       // [nkeys + 1]: next padded index of each bucket
  const int64_t* pad;               // [nkeys + 1][2]: padding lanes [lo, hi) of each bucket
  jgk::JobDev* jobs;
  int32_t* perm;
  uint8_t* vpad;                    // [npad] verdict per padded slot: zeroed for every slot filled
};
void launch_plan_fill(const PlanFillArgs& a, hipStream_t s);

// Stream `bytes` from src to dst with a kernel (16 B per lane where both ends
// are 16-byte aligned, bytes otherwise): the pipeline moves every chunk
// between pinned host memory and HBM this way, through the kernel's own PCIe
// reads / writes, not through the DMA engines (whose command queue stalled
// the host for ~1 ms every few chunks, profiles/r02_pipe_*).
void launch_copy(const void* src, void* dst, size_t bytes, hipStream_t s);

// Zero-copy plans (jg_runtime.cpp, jg_set_zero_copy): copy the token bytes of
// the jobs of one class range [begin, end) from the caller's pinned arena --
// read over PCIe -- into the plan's device arena, key by key at a fixed
// stride per key, and point each job at its copy.  The prep kernels then read
// HBM as in every other path.
struct ZcGatherArgs {
  const uint8_t* src;               // device view of the pinned arena at the plan's base offset
  jgk::JobDev* jobs;                // padded jobs: offsets into src in, into dst out
  int64_t begin, end;               // padded class range
  const uint64_t* kbase;            // per key: byte offset of its region in dst
  const int64_t* kstart;            // per key: first padded slot of its run
  const uint64_t* kstride;          // per key: bytes per slot (a multiple of 16)
  uint8_t* dst;
};
void launch_zc_gather(const ZcGatherArgs& a, hipStream_t s);
