// ganon_ctx.h — internal to libganon_hip.so: the context shared by the masking kernels
// (ganon_hip.hip) and the FASTQ formatter (ganon_fastq.hip), error/launch helpers and the
// per-kernel event timer. Not part of the C ABI (include/ganon.h is).
#ifndef GANON_CTX_H
#define GANON_CTX_H

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <thread>

#include <cstdarg>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

#include "../../include/ganon.h"

struct ganon_inflate_state;                       // ganon_inflate.hip: grow-only device buffers
void ganon_inflate_free(ganon_inflate_state *st);
// ganon_inflate; out == nullptr: the output stays in device memory (ganon_inflate_device_output)
int ganon_inflate_impl(ganon_ctx *ctx, const uint8_t *comp, int64_t comp_len, const int64_t *in_off,
                       const int32_t *in_len, const int64_t *out_off, const int32_t *out_len, int64_t n_blocks,
                       uint8_t *out, int64_t out_total, int64_t *first_bad);

struct ganon_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  bool profiling = false;
  int variant = GANON_VARIANT_DEFAULT;
  int group_unroll = 0;        // GANON_PARAM_GROUP_UNROLL (0 auto: 1 for long reads, else 2)
  int group_skip = 0;          // GANON_PARAM_GROUP_SKIP (profiling only)
  int group_target = 0;        // GANON_PARAM_GROUP_TARGET (0 auto: 704 short reads, 2816 long-read mode), cost units per group (segments + a
                               // per-scope weight of 3: ~512 segments on configs[1], two staging tiles)
  int nt_copy = 1;             // GANON_PARAM_NT_COPY
  int ref2 = 1;                // GANON_PARAM_REF2
  int fq_skip = 0;             // GANON_PARAM_FASTQ_SKIP (profiling only)
  int prep_long = -1;          // GANON_PARAM_PREP_LONG (-1 auto, 0 never, 1 always)
  int fq_kd = 0;               // GANON_PARAM_FASTQ_KD (0: span kernel, 3 units per lane; 16: quad kernel)
  int indel_sort = 0;          // GANON_PARAM_INDEL_SORT
  int group_obs = 0;           // GANON_PARAM_GROUP_OBS (0 auto, 512, 1024)
  int spec_plan = 1;           // GANON_PARAM_SPEC_PLAN (1: speculative replans, 0: every plan synchronizes)
  // the shape of this context's last full plan when a replan of a batch of other sizes may assume it
  // (one-segment mode, no huge scope): its overflow-region entries per incidence and group target
  bool spec_shape_ok = false;
  const void *last_plan = nullptr;   // the batch this context planned last
  int64_t spec_rpi = 0;
  int spec_tgt = 0;
  int prep_unroll = 0;         // GANON_PARAM_PREP_UNROLL (0 auto = 2, 1, 2, 4)
  int far_init = 0;            // GANON_PARAM_FAR_INIT (0 auto)
  int xrec_init = 0;           // GANON_PARAM_XREC_INIT (0 auto)
  int fused_flat = 1;          // GANON_PARAM_FUSED_FLAT (1: one-segment records made in the group kernel)
  bool step_open = false;      // ganon_batch_replan started a profiled step the next run continues
  std::string err;
  struct Rec { std::string name; hipEvent_t e0, e1; };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  std::vector<ganon_kernel_time> last_times;
  // device blocks of released one-shot buffers (FASTQ formatter), reused by size on ctx->stream
  std::multimap<size_t, void *> dcache;
  size_t dcache_bytes = 0;
  ganon_inflate_state *inflate = nullptr;   // BGZF inflate buffers (first ganon_inflate)
  // GANON_INDEL_FORK=1: the indel tally of a batch runs on a side stream forked after the batch's
  // prep (fork_ev, recorded by ganon_batch_run before the group kernel) and joined back (join_ev), so
  // that its latency-bound launches overlap the bandwidth-bound group kernel (they read only the
  // prep's outputs and the raw reads)
  int indel_fork = -1;          // -1: read from the environment at first use
  hipStream_t side = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  const void *fork_db = nullptr;   // the batch fork_ev belongs to (nullptr: none pending)
};

// A device block of at least `bytes` from the context's cache (at most 2x larger), else hipMalloc.
inline hipError_t ctx_dmalloc(ganon_ctx *ctx, void **p, size_t bytes, size_t *got) {
  auto it = ctx->dcache.lower_bound(bytes);
  if (it != ctx->dcache.end() && it->first <= 2 * bytes + (1u << 16)) {
    *p = it->second;
    *got = it->first;
    ctx->dcache_bytes -= it->first;
    ctx->dcache.erase(it);
    return hipSuccess;
  }
  *got = bytes;
  return hipMalloc(p, bytes);
}

// Return a block to the cache (stream order makes its reuse safe: every user runs on ctx->stream),
// or free it when the cache holds 1 GiB already.
inline void ctx_dfree(ganon_ctx *ctx, void *p, size_t bytes) {
  if (!p) return;
  if (ctx && ctx->dcache_bytes + bytes <= (size_t(1) << 30)) {
    ctx->dcache.emplace(bytes, p);
    ctx->dcache_bytes += bytes;
  } else {
    hipFree(p);
  }
}

// Device sequence buffers of an uploaded masking batch (defined in ganon_hip.hip): the input
// (BAM nt16 layout) and the masked output, both `bytes` long.
int ganon_dbatch_seq_buffers(const ganon_dbatch *db, const uint8_t **in, const uint8_t **out, int64_t *bytes);

// Device read/scope arrays of an uploaded masking batch (defined in ganon_hip.hip), for the
// germline indel tally (ganon_indel.hip). read_end = bam_endpos (pos + reference length, or
// pos + 1 for a zero-length alignment).
struct GanonReadView {
  const int32_t *ref_start, *read_len, *read_end, *n_cig, *write_scope;
  const int64_t *seq_off, *cig_off;
  const uint8_t *seq, *dataset;
  const uint32_t *cigar;
  const int64_t *incid_off;
  const int32_t *incid_read;
  const int32_t *span_start, *span_len;
  int32_t n_reads, n_scopes;
};
int ganon_dbatch_read_view(const ganon_dbatch *db, GanonReadView *v);

namespace ganon_detail {

inline int fail(ganon_ctx *ctx, int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  return code;
}

inline hipEvent_t get_event(ganon_ctx *ctx) {
  if (!ctx->pool.empty()) {
    hipEvent_t e = ctx->pool.back();
    ctx->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  hipEventCreate(&e);
  return e;
}

// HIP event pair around the launches of its lifetime when profiling is on
// (ganon_last_kernel_times).
struct KernelScope {
  ganon_ctx *ctx;
  ganon_ctx::Rec rec;
  KernelScope(ganon_ctx *c, const char *name) : ctx(c) {
    if (!ctx->profiling) return;
    rec.name = name;
    rec.e0 = get_event(ctx);
    rec.e1 = get_event(ctx);
    hipEventRecord(rec.e0, ctx->stream);
  }
  ~KernelScope() {
    if (!ctx->profiling) return;
    hipEventRecord(rec.e1, ctx->stream);
    ctx->recs.push_back(rec);
  }
};

inline int check_launch(ganon_ctx *ctx, const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(ctx, GANON_E_DEVICE, "launch of %s failed: %s", what, hipGetErrorString(e));
  // (GANON_SYNC_CHECK=1, debugging only: wait for every checked launch, so that a kernel's fault
  // is reported under its own name)
  static const bool sync_check = [] {
    const char *v = std::getenv("GANON_SYNC_CHECK");
    return v && v[0] == '1';
  }();
  if (sync_check && (e = hipDeviceSynchronize()) != hipSuccess)
    return fail(ctx, GANON_E_DEVICE, "%s failed: %s", what, hipGetErrorString(e));
  return GANON_OK;
}

// Wait for the work queued on stream s without keeping a core busy: an event recorded on s and
// polled with sleeps of 2-100 us. HIP's own waits spin or yield, and with eight processes on one GPU
// (the end-to-end line) the waiting threads took cores from the decode and output threads of the
// GPU's host CPU share. GANON_SLEEP_SYNC=0: hipStreamSynchronize (A/B). One event per host thread
// and device.
inline hipError_t sync_stream(hipStream_t s) {
  static const bool sleepy = [] {
    const char *v = std::getenv("GANON_SLEEP_SYNC");
    return !(v && v[0] == '0');
  }();
  if (!sleepy) return hipStreamSynchronize(s);
  thread_local hipEvent_t ev = nullptr;
  thread_local int ev_dev = -1;
  int dev = 0;
  hipError_t r = hipGetDevice(&dev);
  if (r != hipSuccess) return r;
  if (!ev || ev_dev != dev) {
    if ((r = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return r;
    ev_dev = dev;
  }
  if ((r = hipEventRecord(ev, s)) != hipSuccess) return r;
  unsigned us = 2;
  for (;;) {
    r = hipEventQuery(ev);
    if (r != hipErrorNotReady) return r;
    std::this_thread::sleep_for(std::chrono::microseconds(us));
    us = us < 100 ? 2 * us : 100;
  }
}

// A device-to-host copy into pageable host memory (a status word, a count, a small array): the
// runtime stages such a copy and waits for the stream inside the call, spinning a core while the
// stream's kernels run. The sleep poll waits for the stream first, so the copy finds it idle
// (round 6: the region decoder's readbacks behind the inflate had cost up to 0.5 CPU-s per process
// of the end-to-end line).
inline hipError_t readback(void *dst, const void *src, size_t bytes, hipStream_t s) {
  hipError_t e = sync_stream(s);
  if (e != hipSuccess) return e;
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s);
}

}  // namespace ganon_detail

namespace ganon_wave {

// Inclusive prefix sum over the 64 lanes of a wave (every lane active): DPP row_shr steps inside
// each 16-lane row, then the lower rows' totals through readlane — no LDS crossbar round trips and
// no lane-index arithmetic (a __shfl_up ladder is six ds_bpermute trips per scan). Used by the
// wave-per-read CIGAR walks, where it sits on the critical path of every 64 ops.
__device__ __forceinline__ int incl_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
  const int r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31),
            r2 = __builtin_amdgcn_readlane(v, 47);
  const int row = (int)(threadIdx.x & 63) >> 4;
  return v + (row >= 1 ? r0 : 0) + (row >= 2 ? r1 : 0) + (row >= 3 ? r2 : 0);
}

// The wave's total from an inclusive sum (lane 63), wave-uniform.
__device__ __forceinline__ int last(int incl) { return __builtin_amdgcn_readlane(incl, 63); }

}  // namespace ganon_wave

#define HIP_OR_FAIL(call)                                                                          \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return ganon_detail::fail(ctx, GANON_E_DEVICE, "%s failed: %s", #call, hipGetErrorString(e_)); \
  } while (0)

#endif  // GANON_CTX_H
