// plan.hip — device-side batch planner: groups ESP records by (size class,
// session) so that each 256-record chunk of the GCM kernel has ONE session
// (its GHASH power tables and round keys are staged once in LDS) and records
// of similar length share a wave.  Three small kernels, no host round trip:
//   plan_count     per-workgroup LDS histogram of keys, flushed with one
//                  global atomic per non-empty key per workgroup
//   plan_scan_emit every workgroup: exclusive scan of the key counts ->
//                  record and chunk offsets per key (in LDS), then its range
//                  of the chunk list, one chunk per thread (binary search);
//                  workgroup 0 writes the record cursors and chunk counts
//   plan_scatter   per-workgroup LDS ranks + one global range reservation per
//                  non-empty key -> order[] (a permutation of descriptor
//                  ids); zeroes the counts for the next plan
// Keys: [0, 4*nsas) = GCM records (class-major, largest class first),
// 4*nsas = records with no valid session (chunked with sa = ~0 so the GCM
// kernel marks them EINVAL), 4*nsas+1+s = records of ETA session s.  GCM and
// invalid keys make 256-record (kChunkRecs) chunks, ETA keys 64-record (one wave) chunks;
// chunks are emitted in key order, so nchunks[0] = the GCM kernel's share and
// [nchunks[0], nchunks[1]) the ETA kernel's.  Cost: two passes over the
// 16-byte descriptors.  A session table with more keys than the LDS arrays
// hold takes the same plan through global memory (plan_*_g).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "espgpu_internal.h"

namespace espgpu {

namespace {

constexpr int PWG = 1024;
#ifndef PLAN_PER_THREAD
#define PLAN_PER_THREAD 4
#endif
constexpr int PER_THREAD = PLAN_PER_THREAD;   // records per thread of count / scatter
constexpr int TILE = PWG * PER_THREAD;
constexpr uint32_t kMaxLdsKeys = 16384;   // 64 KiB per LDS array

__device__ __forceinline__ uint32_t size_class(uint32_t len) {
  // GHASH blocks N = ceil((len-32)/16) + 2; steps per lane M = ceil(N/8)
  const int ct = (int)len - 32;
  const int n = (ct > 0 ? (ct + 15) >> 4 : 0) + 2;
  const int m = (n + 7) >> 3;
  return m <= 1 ? 0u : (m <= 4 ? 1u : (m <= 16 ? 2u : 3u));
}

__device__ __forceinline__ uint32_t key_of(const espgpu_desc &d, const DevSA *sas, uint32_t nsas) {
  const uint32_t sa = d.sa;
  if (sa >= nsas) return 4 * nsas;
  const uint32_t mode = sas[sa].mode;
  if (mode == ESPGPU_CSP_MODE_ETA) return 4 * nsas + 1 + sa;
  if (mode != ESPGPU_CSP_MODE_AEAD) return 4 * nsas;
  // largest class first: with the kernels' dynamic chunk queues this is
  // longest-processing-time-first scheduling
  return (3u - size_class(d.len)) * nsas + sa;
}

__host__ __device__ constexpr uint32_t num_keys(uint32_t nsas) { return 5 * nsas + 1; }

__global__ __launch_bounds__(PWG) void plan_count(const espgpu_desc *desc, uint32_t n,
                                                  const DevSA *sas, uint32_t nsas,
                                                  uint32_t *gcnt) {
  __shared__ uint32_t hist[kMaxLdsKeys];
  const uint32_t nkeys = num_keys(nsas);
  for (uint32_t k = threadIdx.x; k < nkeys; k += PWG) hist[k] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * TILE;
#pragma unroll
  for (int j = 0; j < PER_THREAD; ++j) {
    const uint32_t i = base + j * PWG + threadIdx.x;
    if (i < n) atomicAdd(&hist[key_of(desc[i], sas, nsas)], 1u);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < nkeys; k += PWG)
    if (hist[k]) atomicAdd(&gcnt[k], hist[k]);
}

// Chunk cc of the plan: it belongs to the last key whose first chunk is
// <= cc (binary search over the per-key first-chunk offsets coff[0..nkeys],
// coff[nkeys] = the total); roff[k] = key k's first record (roff[nkeys] = n).
// The offsets are in LDS (plan_scan_emit) or, for a session table past the
// LDS arrays, in global memory (plan_emit_g).
template <typename OFF>
__device__ __forceinline__ void emit_chunk(uint32_t cc, const OFF *roff, const OFF *coff, uint32_t nsas,
                                           Chunk *chunks) {
  const uint32_t nkeys = num_keys(nsas), eta0 = 4 * nsas + 1;
  uint32_t lo = 0, hi = nkeys;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (coff[mid] <= cc) lo = mid;
    else hi = mid;
  }
  const uint32_t k = lo, r0 = roff[k], cnt = roff[k + 1] - r0, rpc = k >= eta0 ? 64u : (uint32_t)kChunkRecs;
  const uint32_t sa = k == 4 * nsas ? 0xffffffffu : (k >= eta0 ? k - eta0 : k % nsas);
  const uint32_t cls = k >= 4 * nsas ? 4u : 3u - k / nsas;
  // ceil(cnt / rpc) chunks of EQUAL size (270 records -> 135 + 135, not
  // 256 + 14): a workgroup's pass time grows with its busy waves, so a
  // near-empty remainder chunk costs almost a full pass (cfg2: 1K sessions
  // x 4 size classes leave ~256 +- 16 records per key)
  const uint32_t nc = (cnt + rpc - 1) / rpc, jj = cc - coff[k];
  const uint32_t a = (uint32_t)((uint64_t)cnt * jj / nc), b = (uint32_t)((uint64_t)cnt * (jj + 1) / nc);
  chunks[cc] = Chunk{sa, r0 + a, b - a, cls};
}

// Chunks of key k: 64-record ETA chunks (k >= eta0), 256-record GCM /
// invalid ones (shifts: a run-time divisor was a full integer division per key)
__device__ __forceinline__ uint32_t key_chunks(uint32_t k, uint32_t cnt, uint32_t eta0) {
  static_assert(kChunkRecs == 256, "key_chunks: 256-record GCM chunks");
  return k >= eta0 ? (cnt + 63u) >> 6 : (cnt + 255u) >> 8;
}

// Exclusive scan over the workgroup of each thread's record and chunk
// partials (r, c): within each wave by shuffles, then over the 16 wave
// totals.  Returns the thread's offsets and, to every thread, the totals.
__device__ __forceinline__ void block_scan2(uint32_t r, uint32_t c, uint32_t &roff, uint32_t &coff,
                                            uint32_t &tot_r, uint32_t &tot_c) {
  __shared__ uint32_t s_rec[PWG / 64 + 1], s_chk[PWG / 64 + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t ri = r, ci = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t a = __shfl_up(ri, o), b = __shfl_up(ci, o);
    if (lane >= o) {
      ri += a;
      ci += b;
    }
  }
  if (lane == 63) {
    s_rec[wave] = ri;
    s_chk[wave] = ci;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t ar = 0, ac = 0;
    for (int w = 0; w < PWG / 64; ++w) {
      const uint32_t tr = s_rec[w], tc = s_chk[w];
      s_rec[w] = ar;                       // exclusive wave offsets
      s_chk[w] = ac;
      ar += tr;
      ac += tc;
    }
    s_rec[PWG / 64] = ar;                  // the totals
    s_chk[PWG / 64] = ac;
  }
  __syncthreads();
  roff = s_rec[wave] + ri - r;
  coff = s_chk[wave] + ci - c;
  tot_r = s_rec[PWG / 64];
  tot_c = s_chk[PWG / 64];
}

// The scan and the chunk list in one launch, by every workgroup of
// ceil(max_chunks / PWG): each scans the per-key record and chunk counts
// itself (~5K keys, 5 per thread: cheaper than a launch) into per-key first
// record / first chunk offsets in LDS, then emits the chunks of its range
// (emit_chunk).  Workgroup 0 also writes the record cursors plan_scatter
// advances and the chunk counts the crypto kernels read.  The counts are
// zeroed by plan_scatter, after every workgroup here has read them.
__global__ __launch_bounds__(PWG) void plan_scan_emit(const uint32_t *gcnt, uint32_t nsas, uint32_t *gcur,
                                                      Chunk *chunks, uint32_t *nchunks, uint32_t max_chunks) {
  __shared__ uint32_t s_roff[kMaxLdsKeys + 1], s_coff[kMaxLdsKeys + 1];
  const uint32_t nkeys = num_keys(nsas);
  const uint32_t per = (nkeys + PWG - 1) / PWG;
  const uint32_t k0 = threadIdx.x * per, k1 = min(nkeys, k0 + per);
  const uint32_t eta0 = 4 * nsas + 1;                       // first ETA key
  const bool lead = blockIdx.x == 0;
  // the counts into LDS with coalesced, independent loads (s_roff holds a
  // key's count until its thread replaces it with the key's offset)
  for (uint32_t k = threadIdx.x; k < nkeys; k += PWG) s_roff[k] = gcnt[k];
  __syncthreads();
  uint32_t r = 0, c = 0;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t cnt = s_roff[k];
    r += cnt;
    c += key_chunks(k, cnt, eta0);
  }
  uint32_t roff, coff, tot_r, total;
  block_scan2(r, c, roff, coff, tot_r, total);
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t cnt = s_roff[k];
    s_roff[k] = roff;
    s_coff[k] = coff;
    if (lead) {
      gcur[k] = roff;                      // record cursor (plan_scatter) = the key's first record
      // the GCM kernel's share: the chunks before the first ETA key
      if (k == eta0) nchunks[0] = min(coff, max_chunks);
    }
    roff += cnt;
    coff += key_chunks(k, cnt, eta0);
  }
  if (threadIdx.x == PWG - 1) {
    s_roff[nkeys] = tot_r;
    s_coff[nkeys] = total;
    if (lead) {
      nchunks[1] = min(total, max_chunks);
      if (eta0 >= nkeys) nchunks[0] = min(total, max_chunks);   // no ETA keys (no sessions)
    }
  }
  __syncthreads();
  const uint32_t cc = blockIdx.x * PWG + threadIdx.x;
  if (cc < min(total, max_chunks)) emit_chunk(cc, s_roff, s_coff, nsas, chunks);
}

__global__ __launch_bounds__(PWG) void plan_scatter(const espgpu_desc *desc, uint32_t n,
                                                    const DevSA *sas, uint32_t nsas,
                                                    uint32_t *gcur, uint32_t *order, uint32_t *gcnt) {
  __shared__ uint32_t hist[kMaxLdsKeys], lbase[kMaxLdsKeys];
  const uint32_t nkeys = num_keys(nsas);
  // the counts plan_scan_emit has read, zeroed for the next plan (so the
  // workspace's whole key capacity is zero between plans: no memset)
  for (uint32_t k = blockIdx.x * PWG + threadIdx.x; k < nkeys; k += gridDim.x * PWG) gcnt[k] = 0;
  for (uint32_t k = threadIdx.x; k < nkeys; k += PWG) hist[k] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * TILE;
  uint32_t key[PER_THREAD], rank[PER_THREAD];
#pragma unroll
  for (int j = 0; j < PER_THREAD; ++j) {
    const uint32_t i = base + j * PWG + threadIdx.x;
    key[j] = 0xffffffffu;
    if (i < n) {
      key[j] = key_of(desc[i], sas, nsas);
      rank[j] = atomicAdd(&hist[key[j]], 1u);
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < nkeys; k += PWG)
    if (hist[k]) lbase[k] = atomicAdd(&gcur[k], hist[k]);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER_THREAD; ++j) {
    const uint32_t i = base + j * PWG + threadIdx.x;
    if (i < n) order[lbase[key[j]] + rank[j]] = i;
  }
}

// ---- session tables past the LDS arrays ------------------------------------
// More than kMaxLdsKeys keys (over 3276 sessions): the same plan with the
// per-key arrays in global memory.  Counts and ranks take one global atomic
// per record, a single workgroup scans the counts into groff / gcoff, and the
// chunk list is emitted from those; four launches.  Records of one key land
// in the order their atomics ran, as the LDS ranks of plan_scatter do.
__global__ __launch_bounds__(PWG) void plan_count_g(const espgpu_desc *desc, uint32_t n, const DevSA *sas,
                                                    uint32_t nsas, uint32_t *gcnt) {
  for (uint32_t i = blockIdx.x * PWG + threadIdx.x; i < n; i += gridDim.x * PWG)
    atomicAdd(&gcnt[key_of(desc[i], sas, nsas)], 1u);
}

__global__ __launch_bounds__(PWG) void plan_scan_g(const uint32_t *gcnt, uint32_t nsas, uint32_t *gcur,
                                                   uint32_t *groff, uint32_t *gcoff, uint32_t *nchunks,
                                                   uint32_t max_chunks) {
  const uint32_t nkeys = num_keys(nsas);
  const uint32_t per = (nkeys + PWG - 1) / PWG;
  const uint32_t k0 = threadIdx.x * per, k1 = min(nkeys, k0 + per);
  const uint32_t eta0 = 4 * nsas + 1;
  uint32_t r = 0, c = 0;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t cnt = gcnt[k];
    r += cnt;
    c += key_chunks(k, cnt, eta0);
  }
  uint32_t roff, coff, tot_r, total;
  block_scan2(r, c, roff, coff, tot_r, total);
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t cnt = gcnt[k];
    groff[k] = roff;
    gcoff[k] = coff;
    gcur[k] = roff;
    if (k == eta0) nchunks[0] = min(coff, max_chunks);
    roff += cnt;
    coff += key_chunks(k, cnt, eta0);
  }
  if (threadIdx.x == PWG - 1) {
    groff[nkeys] = tot_r;
    gcoff[nkeys] = total;
    nchunks[1] = min(total, max_chunks);
    if (eta0 >= nkeys) nchunks[0] = min(total, max_chunks);
  }
}

__global__ __launch_bounds__(PWG) void plan_emit_g(const uint32_t *groff, const uint32_t *gcoff, uint32_t nsas,
                                                   Chunk *chunks, uint32_t max_chunks) {
  const uint32_t cc = blockIdx.x * PWG + threadIdx.x;
  if (cc < min(gcoff[num_keys(nsas)], max_chunks)) emit_chunk(cc, groff, gcoff, nsas, chunks);
}

__global__ __launch_bounds__(PWG) void plan_scatter_g(const espgpu_desc *desc, uint32_t n, const DevSA *sas,
                                                      uint32_t nsas, uint32_t *gcur, uint32_t *order,
                                                      uint32_t *gcnt) {
  const uint32_t nkeys = num_keys(nsas);
  for (uint32_t k = blockIdx.x * PWG + threadIdx.x; k < nkeys; k += gridDim.x * PWG) gcnt[k] = 0;
  for (uint32_t i = blockIdx.x * PWG + threadIdx.x; i < n; i += gridDim.x * PWG)
    order[atomicAdd(&gcur[key_of(desc[i], sas, nsas)], 1u)] = i;
}

}  // namespace

// gcnt, gcur: one word per key; groff, gcoff (the global-memory plan past
// kMaxLdsKeys keys): one more
size_t plan_workspace_words(uint32_t nsas) { return 4 * (size_t)num_keys(nsas) + 2; }
uint32_t plan_max_chunks(uint32_t n, uint32_t nsas) { return n / 64 + num_keys(nsas) + 8; }

int launch_plan(const espgpu_desc *d_desc, uint32_t n, const DevSA *sas, uint32_t nsas, uint32_t cap_sas,
                uint32_t *d_work, uint32_t *d_order, Chunk *d_chunks, uint32_t *d_nchunks,
                uint32_t max_chunks, void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t nkeys = num_keys(nsas);
  if (nsas > cap_sas) return -1;
  // gcnt is zero on entry (plan_scatter re-zeroes it) over the workspace's whole
  // key capacity; the cursors sit after that capacity, not after this batch's
  // keys: the key count grows with the session table, and cursor words left
  // where a later batch's counts go would be counted
  const uint32_t capk = num_keys(cap_sas);
  uint32_t *gcnt = d_work, *gcur = d_work + capk;
  if (nkeys > kMaxLdsKeys) {
    uint32_t *groff = gcur + capk, *gcoff = groff + capk + 1;
    const uint32_t g = std::min<uint32_t>((n + PWG - 1) / PWG, 2048);
    if (g) hipLaunchKernelGGL(plan_count_g, dim3(g), dim3(PWG), 0, st, d_desc, n, sas, nsas, gcnt);
    hipLaunchKernelGGL(plan_scan_g, dim3(1), dim3(PWG), 0, st, gcnt, nsas, gcur, groff, gcoff, d_nchunks,
                       max_chunks);
    hipLaunchKernelGGL(plan_emit_g, dim3((max_chunks + PWG - 1) / PWG), dim3(PWG), 0, st, groff, gcoff, nsas,
                       d_chunks, max_chunks);
    hipLaunchKernelGGL(plan_scatter_g, dim3(std::max<uint32_t>(g, (nkeys + PWG - 1) / PWG)), dim3(PWG), 0, st,
                       d_desc, n, sas, nsas, gcur, d_order, gcnt);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const uint32_t grid = (n + TILE - 1) / TILE;
  if (grid) hipLaunchKernelGGL(plan_count, dim3(grid), dim3(PWG), 0, st, d_desc, n, sas, nsas, gcnt);
  hipLaunchKernelGGL(plan_scan_emit, dim3((max_chunks + PWG - 1) / PWG), dim3(PWG), 0, st, gcnt, nsas, gcur,
                     d_chunks, d_nchunks, max_chunks);
  if (grid) hipLaunchKernelGGL(plan_scatter, dim3(grid), dim3(PWG), 0, st, d_desc, n, sas, nsas, gcur,
                               d_order, gcnt);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace espgpu
