// plan.hip — device-side batch planner: groups ESP records by (size class,
// session) so that each 256-record chunk of the GCM kernel has ONE session
// (its GHASH power tables and round keys are staged once in LDS) and records
// of similar length share a wave.  Three small kernels, no host round trip:
//   plan_count   per-workgroup LDS histogram of keys, flushed with one global
//                atomic per non-empty key per workgroup
//   plan_scan    one workgroup: exclusive scan of key counts -> record offsets
//                and chunk offsets; writes the chunk list and its length
//   plan_scatter per-workgroup LDS ranks + one global range reservation per
//                non-empty key -> order[] (a permutation of descriptor ids)
// Keys: [0, 4*nsas) = GCM records (class-major, largest class first),
// 4*nsas = records with no valid session (chunked with sa = ~0 so the GCM
// kernel marks them EINVAL), 4*nsas+1+s = records of ETA session s.  GCM and
// invalid keys make 256-record (kChunkRecs) chunks, ETA keys 64-record (one wave) chunks;
// chunks are emitted in key order, so nchunks[0] = the GCM kernel's share and
// [nchunks[0], nchunks[1]) the ETA kernel's.  Cost: two passes over the
// 16-byte descriptors.
#include <hip/hip_runtime.h>

#include "espgpu_internal.h"

namespace espgpu {

namespace {

constexpr int PWG = 1024;
constexpr int PER_THREAD = 4;
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

// Single workgroup.  gcnt[nkeys] -> gcur[nkeys] (record cursor), chunks.
// Scan of the per-key record and chunk counts (each thread sums a run of
// keys, Hillis-Steele over the 1024 partials), per-key offsets into LDS,
// then every thread emits chunks c = tid, tid + 1024, ...: the key of chunk c
// is the last key whose first chunk is <= c (binary search in LDS), so the
// chunk list is written evenly by all threads whatever the key sizes.  (The
// kernel takes ~33 us for 1K ETA sessions either way; the serial per-thread
// emission it replaced was not its cost.)
__global__ __launch_bounds__(PWG) void plan_scan(const uint32_t *gcnt, uint32_t nsas,
                                                 uint32_t *gcur, Chunk *chunks,
                                                 uint32_t *nchunks, uint32_t max_chunks) {
  __shared__ uint32_t s_rec[PWG], s_chk[PWG];
  // per key: first chunk, first record (s_roff[nkeys] = all records)
  __shared__ uint32_t s_coff[kMaxLdsKeys], s_roff[kMaxLdsKeys + 1];
  const uint32_t nkeys = num_keys(nsas);
  const uint32_t per = (nkeys + PWG - 1) / PWG;
  const uint32_t k0 = threadIdx.x * per, k1 = min(nkeys, k0 + per);
  const uint32_t eta0 = 4 * nsas + 1;                       // first ETA key
  auto recs_per_chunk = [&](uint32_t k) { return k >= eta0 ? 64u : (uint32_t)kChunkRecs; };
  uint32_t r = 0, c = 0;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t cnt = gcnt[k];
    r += cnt;
    c += (cnt + recs_per_chunk(k) - 1) / recs_per_chunk(k);
  }
  s_rec[threadIdx.x] = r;
  s_chk[threadIdx.x] = c;
  __syncthreads();
  for (int o = 1; o < PWG; o <<= 1) {
    uint32_t a = threadIdx.x >= (unsigned)o ? s_rec[threadIdx.x - o] : 0;
    uint32_t b = threadIdx.x >= (unsigned)o ? s_chk[threadIdx.x - o] : 0;
    __syncthreads();
    s_rec[threadIdx.x] += a;
    s_chk[threadIdx.x] += b;
    __syncthreads();
  }
  uint32_t roff = s_rec[threadIdx.x] - r, coff = s_chk[threadIdx.x] - c;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t cnt = gcnt[k];
    gcur[k] = roff;                       // record cursor (plan_scatter) = the key's first record
    s_roff[k] = roff;
    s_coff[k] = coff;
    roff += cnt;
    coff += (cnt + recs_per_chunk(k) - 1) / recs_per_chunk(k);
  }
  if (threadIdx.x == PWG - 1) s_roff[nkeys] = s_rec[PWG - 1];
  __syncthreads();
  const uint32_t total = s_chk[PWG - 1];
  if (threadIdx.x == 0) {
    nchunks[1] = min(total, max_chunks);
    // the GCM kernel's share: the chunks before the first ETA key
    nchunks[0] = eta0 < nkeys ? min(s_coff[eta0], max_chunks) : nchunks[1];
  }
  const uint32_t lim = min(total, max_chunks);
  for (uint32_t ci = threadIdx.x; ci < lim; ci += PWG) {
    uint32_t lo = 0, hi = nkeys;                          // last key with s_coff <= ci
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_coff[mid] <= ci) lo = mid;
      else hi = mid;
    }
    const uint32_t k = lo, cnt = s_roff[k + 1] - s_roff[k], rpc = recs_per_chunk(k);
    const uint32_t sa = k == 4 * nsas ? 0xffffffffu : (k >= eta0 ? k - eta0 : k % nsas);
    const uint32_t cls = k >= 4 * nsas ? 4u : 3u - k / nsas;
    // ceil(cnt / rpc) chunks of EQUAL size (270 records -> 135 + 135, not
    // 256 + 14): a workgroup's pass time grows with its busy waves, so a
    // near-empty remainder chunk costs almost a full pass (cfg2: 1K sessions
    // x 4 size classes leave ~256 +- 16 records per key)
    const uint32_t nc = (cnt + rpc - 1) / rpc, jj = ci - s_coff[k];
    const uint32_t a = (uint32_t)((uint64_t)cnt * jj / nc), b = (uint32_t)((uint64_t)cnt * (jj + 1) / nc);
    chunks[ci] = Chunk{sa, s_roff[k] + a, b - a, cls};
  }
}

__global__ __launch_bounds__(PWG) void plan_scatter(const espgpu_desc *desc, uint32_t n,
                                                    const DevSA *sas, uint32_t nsas,
                                                    uint32_t *gcur, uint32_t *order) {
  __shared__ uint32_t hist[kMaxLdsKeys], lbase[kMaxLdsKeys];
  const uint32_t nkeys = num_keys(nsas);
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

}  // namespace

// gcnt[nkeys] + gcur[nkeys]
size_t plan_workspace_words(uint32_t nsas) { return 2 * (size_t)num_keys(nsas); }
uint32_t plan_max_chunks(uint32_t n, uint32_t nsas) { return n / 64 + num_keys(nsas) + 8; }

int launch_plan(const espgpu_desc *d_desc, uint32_t n, const DevSA *sas, uint32_t nsas,
                uint32_t *d_work, uint32_t *d_order, Chunk *d_chunks, uint32_t *d_nchunks,
                uint32_t max_chunks, void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t nkeys = num_keys(nsas);
  if (nkeys > kMaxLdsKeys) return -1;     // caller must pre-group (ESPGPU_BATCH_GROUPED)
  uint32_t *gcnt = d_work, *gcur = d_work + nkeys;
  if (hipMemsetAsync(gcnt, 0, nkeys * sizeof(uint32_t), st) != hipSuccess) return -1;
  const uint32_t grid = (n + TILE - 1) / TILE;
  if (grid) hipLaunchKernelGGL(plan_count, dim3(grid), dim3(PWG), 0, st, d_desc, n, sas, nsas, gcnt);
  hipLaunchKernelGGL(plan_scan, dim3(1), dim3(PWG), 0, st, gcnt, nsas, gcur, d_chunks, d_nchunks,
                     max_chunks);
  if (grid) hipLaunchKernelGGL(plan_scatter, dim3(grid), dim3(PWG), 0, st, d_desc, n, sas, nsas, gcur,
                               d_order);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace espgpu
