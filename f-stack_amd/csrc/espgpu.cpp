// espgpu.cpp — host runtime behind include/espgpu.h: the opencrypto-driver
// shaped C ABI (sessions, process/flush/poll with pinned staging and async
// copies on a HIP stream) and the device-resident batch entry points.
//
// Reference interfaces mirrored (F-Stack 1.25 tree):
//   probesession  freebsd/opencrypto/cryptosoft.c:1244-1303 (swcr_probesession)
//                 + check_csp, freebsd/opencrypto/crypto.c:746-870
//   newsession    cryptosoft.c:1309-1409, swcr_setup_gcm :1087, _cipher :976, _auth :1003
//   freesession   cryptosoft.c:1412
//   process       cryptosoft.c:1429-1441 (swcr_process) -> swcr_gcm :465 / swcr_eta :874
//   completion    crypto_done, crypto.c:1802
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "espgpu.h"
#include "espgpu_internal.h"
#include "fifo_arena.h"
#include "host_crypto.h"

using namespace espgpu;

namespace {

#ifndef GCM_BURST_DEFAULT
#define GCM_BURST_DEFAULT 4096
#endif
#ifndef GPU_TIME_SMALL
#define GPU_TIME_SMALL 0
#endif
// flush(): batches up to this many staged bytes run on one stream (latency)
constexpr uint32_t kSmallBatchBytes = 128u << 10;

struct Session {
  bool used = false;
  int mode = 0, flags = 0, mlen = 0, klen = 0;
  bool ctr = false;       // ETA / CIPHER with AES-ICM (RFC 3686 ESP AES-CTR)
  bool null = false;      // ETA / CIPHER with CRYPTO_NULL_CBC (ESP-NULL)
  bool whash = false;     // HMAC-SHA2-384/512 (128-byte hash blocks)
  bool wide = false;      // served by the two-pass ETA kernels only: HMAC-SHA2-384/512
                          // (128-byte hash blocks), no auth (CIPHER) or ESP-NULL
};

struct Pending {
  void *opaque;
  int etype_pre;              // -1: take the device status; else a host-side errno
  uint32_t rec;               // descriptor index in the batch
  uint32_t stage_off;         // byte offset of the staged record
  uint32_t stage_len;
  // where the result bytes go back: [buf_off, buf_off+n) of the request buffer
  // receives staged bytes [stage_from, stage_from+n); up to 2 spans
  struct Span { uint32_t buf_off, stage_from, n; } span[2];
  int nspan;
  uint32_t seg0, nsegs;       // the request's segments, copied into Slot::segpool
  // zero-copy: the record's start in registered host memory (device-mapped
  // address, espgpu_register_host); 0 = gathered into the staging buffer.
  // The record's layout there is the staged one, so span k's bytes go to
  // zc + span[k].stage_from.
  uint64_t zc;
};

// A request process() accepted while every staging slot was in flight
// (set_tuning "overflow_mb"): its bytes (unless zero-copy) wait in host
// memory and flush() moves it into the next free slot, in arrival order.
struct OvfEntry {
  Pending pd;                 // stage_off / seg0 index the overflow's own buffers
  espgpu_desc d;
  int32_t sid;
  uint8_t op, kind;
};
// The host overflow: entries in a fixed ring, their gathered bytes and segment
// lists in fixed FIFO arenas (fifo_arena.h), all sized at
// set_tuning("overflow_mb").
struct Overflow {
  std::unique_ptr<OvfEntry[]> ent;
  size_t ecap = 0, head = 0, count = 0;   // ring of entries; head = oldest
  FifoArena<uint8_t> bytes;
  FifoArena<espgpu_seg> segpool;
  size_t live_bytes = 0, peak_bytes = 0;
  bool empty() const { return count == 0; }
  OvfEntry &front() { return ent[head]; }
  // Reserve the three rings (the overflow must be empty).  All or nothing:
  // false leaves the old rings in place (the caller answers ENOMEM; no
  // exception crosses the C ABI).
  bool init(size_t cap_bytes) {
    // the byte ring holds overflow_mb of records; entries (a zero-copy record
    // needs no bytes) and segment lists get rings of their own beside it
    const size_t ne = cap_bytes ? std::max<size_t>(256, std::min<size_t>(cap_bytes / 512, (size_t)1 << 22)) : 0;
    std::unique_ptr<OvfEntry[]> e(ne ? new (std::nothrow) OvfEntry[ne] : nullptr);
    FifoArena<uint8_t> b;
    FifoArena<espgpu_seg> sg;
    if ((ne && !e) || !b.init(cap_bytes) || !sg.init(ne * 4)) return false;
    // the entry ring's pages committed now too, as the arenas' (fifo_arena.h)
    for (size_t o = 0; o < ne * sizeof(OvfEntry); o += 4096)
      reinterpret_cast<volatile uint8_t *>(e.get())[o] = 0;
    ent.swap(e);
    ecap = ne;
    bytes.swap(b);
    segpool.swap(sg);
    head = count = 0;
    live_bytes = peak_bytes = 0;
    return true;
  }
  size_t reserved() const {
    return ecap * sizeof(OvfEntry) + bytes.cap + segpool.cap * sizeof(espgpu_seg);
  }
  void pop() {
    OvfEntry &e = ent[head];
    if (!e.pd.zc) bytes.pop(e.pd.stage_off, (e.pd.stage_len + 15) & ~15u);
    segpool.pop(e.pd.seg0, e.pd.nsegs);
    live_bytes -= e.pd.zc ? 0 : ((e.pd.stage_len + 15) & ~15u);
    head = (head + 1) % ecap;
    if (--count == 0) {
      head = 0;
      bytes.clear();
      segpool.clear();
    }
  }
};

// Host memory registered with espgpu_register_host.
struct HostRegion {
  uintptr_t base;
  uint64_t len;
  uint64_t dev;               // device-mapped address of base
  bool owned;                 // hipHostRegister'ed here (else already pinned)
};

enum { SLOT_FREE = 0, SLOT_FILLING = 1, SLOT_INFLIGHT = 2 };

// A staging slot.  One pinned host buffer and its device mirror(s) hold, at
// flush time, [records: bytes][16 B slack][descriptors: nrec*16][status: nrec],
// so a batch is ONE H2D copy, the kernel(s), and ONE D2H copy (records and
// status together) -- what bounds a 32-record burst's latency is the number of
// queue operations, not bytes.
struct Slot {
  int state = SLOT_FREE;
  int op = -1;                // 0 decrypt, 1 encrypt
  uint8_t *h_arena = nullptr, *d_arena = nullptr, *d_out = nullptr;
  uint8_t *h_arena_dev = nullptr;           // h_arena's device-mapped address (xfer kernel)
  espgpu_desc *h_desc = nullptr;            // descriptors while filling
  // the xfer kernel's span lists (pinned, read by the kernel through the
  // mapping): [0, nin) before the crypto kernels, [nin, nin + nout) after
  XferSpan *h_xfer = nullptr, *h_xfer_dev = nullptr;
  uint32_t xfer_cap = 0;
  uint32_t nrec = 0, bytes = 0;
  uint32_t nstaged = 0;                     // records gathered (not zero-copy)
  uint32_t desc_off = 0, stat_off = 0;      // set by flush
  int32_t sid0 = -1;                        // session of the first record
  bool mixed = false;                       // more than one session staged
  uint32_t kinds = 0;                       // 1: GCM records, 2: ETA records
  std::vector<Pending> reqs;             // reserved to batch_records: no per-record allocation
  std::vector<espgpu_seg> segpool;       // segment lists of the staged requests
  hipEvent_t in_done = nullptr, k0 = nullptr, k1 = nullptr, kout = nullptr, done = nullptr;
  bool timed = false;                       // k0 / k1 recorded around the kernels
  hipStream_t st = nullptr;                 // small batches: copy, kernel, copy in order here
  // doorbell path (set_tuning "door"): the job number this slot's batch was
  // published as (-1: launched, or free), when, and its own E_K(J0) scratch
  // (jobs of different slots run at once)
  int64_t door_job = -1;
  uint64_t door_t0 = 0;
  uint4 *d_ej0 = nullptr;
  uint64_t t_launch = 0;                    // host clock (ns) when the batch was launched / published
  bool stuck = false;                       // fault injection: its completion is never seen (set_tuning "fault" 4)
  hipStream_t wq = nullptr;                 // launch in progress: the stream host-writing work went to
};

}  // namespace

struct espgpu_ctx {
  int device = 0;
  espgpu_config cfg{};
  // three streams so that batch k+1's H2D, batch k's kernels and batch k-1's
  // D2H overlap: stream (compute), s_in (host->device), s_out (device->host)
  hipStream_t stream = nullptr, s_in = nullptr, s_out = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // host-to-host pipeline (espgpu_decrypt_host) device mirrors
  uint8_t *e2e_arena = nullptr, *e2e_out = nullptr, *e2e_status = nullptr;
  espgpu_desc *e2e_desc = nullptr;
  uint64_t e2e_bytes = 0;
  uint32_t e2e_n = 0;
  hipEvent_t e2e_in[2] = {nullptr, nullptr}, e2e_k[2] = {nullptr, nullptr};
  DevSA *d_sas = nullptr;
  uint8_t *d_gtab = nullptr;
  uint2 *d_tpair = nullptr, *d_dpair = nullptr;
  uint8_t *d_isbox = nullptr;
  uint32_t *d_queue = nullptr;   // work-queue regions (kQueueRegionWords apart): GCM, ETA, ETA aux (self-resetting)
  std::vector<Session> sessions;
  std::vector<DevSA> h_sas;
  // ETA sessions: all, and by kernel: narrow-hash (SHA-1 / SHA2-256) CBC and
  // CTR, wide-hash (SHA2-384/512) CBC and CTR
  int n_eta = 0, n_cbc = 0, n_ctr = 0, n_wcbc = 0, n_wctr = 0;
  int n_gcm = 0;                 // live AEAD (GCM) sessions
  bool plan_dirty = true;        // planner key counts not known to be zero (plan_scan re-zeroes them)
  int n_whash = 0;   // ETA sessions with HMAC-SHA2-384/512 (the wide-hash two-pass kernels)
  // GCM lanes per record: 0 = by batch size, 4 or 8 forced (set_tuning
  // "gcm_lanes": the tests run both kernels at every batch size)
  int gcm_lanes = 0;
  // E_K(J0) scratch of the burst kernel
  uint4 *d_ej0 = nullptr;
  uint32_t ej0_cap = 0;
  // planner workspace
  uint32_t plan_cap = 0;
  uint32_t *d_work = nullptr, *d_order = nullptr, *d_nchunks = nullptr;
  Chunk *d_chunks = nullptr;
  uint32_t max_chunks = 0;
  // staging
  std::vector<Slot> slots;
  int cur = 0;
  Overflow ovf;
  size_t ovf_cap = 0;            // set_tuning "overflow_mb" (0: ERESTART when the slots are busy)
  int xfer_small = 1;            // small batches: staging region moved by the xfer kernel (else hipMemcpyAsync)
  int stage_fused = 1;           // small single-session GCM batches stage their own records (one launch)
  uint32_t gcm_burst = GCM_BURST_DEFAULT;   // small GCM batches of <= this many records: burst kernel
  // doorbell burst path (set_tuning "door", espgpu_internal.h DoorCtl): a
  // persistent kernel of door_wg workgroups serves single-session GCM
  // batches of <= gcm_burst records with no launch per batch
  int door_wg = 0;
  uint32_t door_idle_us = 20000;             // the kernel exits after this long without a job
  bool door_retiring = false;                // kDoorStopIdle requested (door_retire)
  DoorCtl *door_ctl = nullptr, *door_ctl_dev = nullptr;
  DoorDev *d_door = nullptr;
  DoorSlot *d_door_slots = nullptr;
  hipStream_t s_door = nullptr;
  hipEvent_t ev_door = nullptr;
  bool door_live = false;                    // launched and not seen to have exited
  uint32_t door_next = 0;                    // next job number
  uint64_t door_last_pub = 0;                // host clock (ns) of the last publish
  std::vector<HostRegion> regions;   // sorted by base
  // completions not yet handed to poll(): ready[ready_head..] (host-side
  // rejects and finished batches), reserved so steady state does not allocate
  std::vector<espgpu_completion> ready;
  size_t ready_head = 0;
  // the stream the ctx last launched on and an event after that launch: the
  // work-queue counters and planner workspace are per ctx, so a launch on a
  // different stream first waits for it (stream-ordered, never concurrent)
  hipStream_t last_st = nullptr;
  bool launched = false;
  hipEvent_t ev_last = nullptr;
  // GPU failure (ctx_fail): once set the ctx launches nothing again; every
  // request it holds completes exactly once with ESPGPU_EIO
  bool failed = false;
  uint32_t fault = 0;            // set_tuning "fault": injected failures (ESPGPU_FAULT_*)
  uint32_t deadline_ms = 2000;   // set_tuning "deadline_ms": a batch outstanding this long is a GPU failure
  espgpu_stats stats{};
  float last_ms = 0.f;
  std::string err;
};

namespace {

int fail(espgpu_ctx *c, int code, const char *fmt, ...) {
  if (c) {
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define HIPCHK(ctx, expr)                                                          \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) return fail(ctx, ESPGPU_EIO, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }
uint32_t ror16(uint32_t v) { return (v >> 16) | (v << 16); }

// The ETA-kernel session counter a session belongs to: which decrypt and
// cipher-pass kernels a batch may need (launch_eta kinds).  ESP-NULL sessions
// need no cipher pass; they count as CTR so that no CBC pass is launched.
int &eta_count(espgpu_ctx *c, const Session &s) {
  const bool ctr = s.ctr || s.null;
  return s.wide ? (ctr ? c->n_wctr : c->n_wcbc) : (ctr ? c->n_ctr : c->n_cbc);
}

int ensure_plan(espgpu_ctx *c, uint32_t n) {
  const uint32_t need_chunks = plan_max_chunks(n, c->cfg.max_sessions);
  if (n <= c->plan_cap && need_chunks <= c->max_chunks) return 0;
  hipFree(c->d_work);
  hipFree(c->d_order);
  hipFree(c->d_chunks);
  hipFree(c->d_nchunks);
  c->plan_cap = std::max(n, 1024u);
  c->max_chunks = plan_max_chunks(c->plan_cap, c->cfg.max_sessions);
  // key histograms sized for the SA table's capacity: sessions created after
  // this allocation must not outgrow it
  HIPCHK(c, hipMalloc(&c->d_work, plan_workspace_words(c->cfg.max_sessions) * 4));
  HIPCHK(c, hipMalloc(&c->d_order, (size_t)c->plan_cap * 4));
  HIPCHK(c, hipMalloc(&c->d_chunks, (size_t)c->max_chunks * sizeof(Chunk)));
  HIPCHK(c, hipMalloc(&c->d_nchunks, 16));
  c->plan_dirty = true;
  return 0;
}

// Copy `n` bytes at logical offset `off` of a segmented buffer.
bool seg_copy_out(const espgpu_seg *segs, uint32_t nsegs, uint32_t off, uint32_t n, uint8_t *dst) {
  for (uint32_t i = 0; i < nsegs; ++i) {
    const espgpu_seg &s = segs[i];
    if (off >= s.len) { off -= s.len; continue; }
    uint32_t k = std::min(n, s.len - off);
    memcpy(dst, (const uint8_t *)s.base + off, k);
    dst += k; n -= k; off = 0;
    if (!n) return true;
  }
  return n == 0;
}
bool seg_copy_in(const espgpu_seg *segs, uint32_t nsegs, uint32_t off, uint32_t n, const uint8_t *src) {
  for (uint32_t i = 0; i < nsegs; ++i) {
    const espgpu_seg &s = segs[i];
    if (off >= s.len) { off -= s.len; continue; }
    uint32_t k = std::min(n, s.len - off);
    memcpy((uint8_t *)s.base + off, src, k);
    src += k; n -= k; off = 0;
    if (!n) return true;
  }
  return n == 0;
}

int alloc_slot(espgpu_ctx *c, Slot &s) {
  const size_t recs = c->cfg.batch_records;
  const size_t bytes = c->cfg.batch_bytes + 64 + recs * (sizeof(espgpu_desc) + 1) + 64;
  HIPCHK(c, hipHostMalloc((void **)&s.h_arena, bytes, hipHostMallocDefault));
  HIPCHK(c, hipHostGetDevicePointer((void **)&s.h_arena_dev, s.h_arena, 0));
  s.h_desc = new espgpu_desc[recs];
  HIPCHK(c, hipMalloc(&s.d_arena, bytes));
  HIPCHK(c, hipMalloc(&s.d_out, bytes));
  HIPCHK(c, hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  HIPCHK(c, hipEventCreateWithFlags(&s.in_done, hipEventDisableTiming));
  HIPCHK(c, hipEventCreate(&s.k0));
  HIPCHK(c, hipEventCreate(&s.k1));
  HIPCHK(c, hipEventCreateWithFlags(&s.kout, hipEventDisableTiming));
  HIPCHK(c, hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking));
  s.reqs.reserve(recs);
  s.segpool.reserve(recs * 2);
  return 0;
}

void free_slot(Slot &s) {
  if (s.st) hipStreamSynchronize(s.st);
  hipHostFree(s.h_arena);
  hipHostFree(s.h_xfer);
  hipFree(s.d_ej0);
  delete[] s.h_desc;
  hipFree(s.d_arena); hipFree(s.d_out);
  for (hipEvent_t e : {s.done, s.in_done, s.k0, s.k1, s.kout})
    if (e) hipEventDestroy(e);
  if (s.st) hipStreamDestroy(s.st);
}

// The device-mapped address of [p, p + n) if it lies in one registered region, else 0.
uint64_t region_dev(const espgpu_ctx *c, const uint8_t *p, uint32_t n) {
  const uintptr_t a = (uintptr_t)p;
  auto it = std::upper_bound(c->regions.begin(), c->regions.end(), a,
                             [](uintptr_t v, const HostRegion &r) { return v < r.base; });
  if (it == c->regions.begin()) return 0;
  --it;
  if (a + n > it->base + it->len) return 0;
  return it->dev + (a - it->base);
}

// [off, off + n) of a segmented buffer if it lies in one segment, else nullptr.
const uint8_t *seg_span(const espgpu_seg *segs, uint32_t nsegs, uint32_t off, uint32_t n) {
  for (uint32_t i = 0; i < nsegs; ++i) {
    if (off >= segs[i].len) { off -= segs[i].len; continue; }
    return off + n <= segs[i].len ? (const uint8_t *)segs[i].base + off : nullptr;
  }
  return nullptr;
}

// Append one request to a slot (its record bytes, unless zero-copy, already
// at h_arena + bytes).
void slot_commit(Slot &s, Pending pd, espgpu_desc d, const espgpu_seg *segs, int32_t sid, int op,
                 uint32_t kind) {
  if (s.state == SLOT_FREE) {
    s.state = SLOT_FILLING;
    s.op = op;
    s.nrec = 0;
    s.bytes = 0;
    s.nstaged = 0;
    s.reqs.clear();
    s.segpool.clear();
    s.sid0 = sid;
    s.mixed = false;
    s.kinds = 0;
  }
  pd.rec = s.nrec;
  pd.stage_off = s.bytes;
  pd.seg0 = (uint32_t)s.segpool.size();
  s.segpool.insert(s.segpool.end(), segs, segs + pd.nsegs);
  d.off4 = s.bytes / 4;
  s.h_desc[s.nrec] = d;
  s.bytes += (pd.stage_len + 15) & ~15u;
  s.nrec++;
  s.nstaged += pd.zc ? 0 : 1;
  s.mixed |= (sid != s.sid0);
  s.kinds |= kind;
  s.reqs.push_back(pd);
}

bool slot_full(const espgpu_ctx *c, const Slot &s, int op, uint32_t rlen) {
  return s.state == SLOT_FILLING &&
         (s.op != op || s.nrec >= c->cfg.batch_records || s.bytes + rlen + 16 > c->cfg.batch_bytes);
}

uint64_t now_ns() {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

// ---- doorbell burst path (espgpu_internal.h DoorCtl) -------------------------
// A door batch's descriptors and statuses sit at fixed offsets of its slot
// (after the largest record region), so the device slot table never changes
// per batch; its xout spans start at h_xfer + batch_records.
uint32_t door_desc_off(const espgpu_ctx *c) { return c->cfg.batch_bytes + 16; }
uint32_t door_stat_off(const espgpu_ctx *c) { return door_desc_off(c) + c->cfg.batch_records * (uint32_t)sizeof(espgpu_desc); }
constexpr uint32_t kDoorChunk = 4;           // records per claimed chunk (the burst kernel's)

int door_write_slot(espgpu_ctx *c, size_t k) {
  const Slot &s = c->slots[k];
  const DoorSlot ds{s.d_arena, s.d_out, s.d_ej0, s.h_xfer_dev, s.h_xfer_dev + c->cfg.batch_records,
                    s.h_arena_dev + door_desc_off(c), s.h_arena_dev + door_stat_off(c), door_desc_off(c),
                    door_stat_off(c)};
  HIPCHK(c, hipMemcpy(c->d_door_slots + k, &ds, sizeof ds, hipMemcpyHostToDevice));
  return 0;
}

// The kernel has exited (or was never launched): no workgroup reads the
// slot table or the SA table's cached state any more.
bool door_exited(espgpu_ctx *c) {
  // (an error other than "not ready": the device is gone, and so is the kernel)
  if (c->door_live && hipEventQuery(c->ev_door) != hipErrorNotReady) c->door_live = false;
  return !c->door_live;
}

// Stop the persistent kernel and wait for it (published jobs it did not
// claim stay in the ring for the next launch).  A failed ctx only asks: its
// kernel may never finish, and nothing waits on a failed device.
void door_stop(espgpu_ctx *c) {
  if (!c->door_live) return;
  __atomic_store_n(&c->door_ctl->stop, kDoorStopNow, __ATOMIC_SEQ_CST);
  if (c->failed) return;
  hipEventSynchronize(c->ev_door);
  __atomic_store_n(&c->door_ctl->stop, 0u, __ATOMIC_SEQ_CST);
  c->door_live = false;
  c->door_retiring = false;
}

// Before any other kernel or copy of this ctx is queued: the persistent
// kernel's stream may share a hardware queue with the stream that work goes
// to (GPU_MAX_HW_QUEUES is 4; a ctx has more streams), and a queue runs its
// packets in order, so work behind a resident door kernel would wait for its
// idle timeout.  Without waiting, ask it to exit once no published job is
// left (kDoorStopIdle): queued work starts right after its last chunk.  The
// next door job clears the request and relaunches the kernel if it exited.
void door_retire(espgpu_ctx *c) {
  if (!c->door_live || c->door_retiring) return;
  if (door_exited(c)) return;
  __atomic_store_n(&c->door_ctl->stop, kDoorStopIdle, __ATOMIC_SEQ_CST);
  c->door_retiring = true;
}

// No launched work of the ctx is outstanding: its last launch (any stream)
// and every launched slot's batch have completed.  Until then a retire
// request must stand: the launched work may sit behind the door kernel on a
// shared hardware queue.
bool launched_idle(espgpu_ctx *c) {
  if (c->launched && hipEventQuery(c->ev_last) != hipSuccess) return false;
  for (const Slot &s : c->slots)
    if (s.state == SLOT_INFLIGHT && s.door_job < 0 && hipEventQuery(s.done) != hipSuccess) return false;
  return true;
}

int door_launch(espgpu_ctx *c) {
  DoorArgs a{};
  a.ctl = c->door_ctl_dev;
  a.dev = c->d_door;
  a.slots = c->d_door_slots;
  a.nslots = (uint32_t)c->slots.size();
  a.chunk = kDoorChunk;
  a.idle_ticks = c->door_idle_us * 100u;     // s_memrealtime: 100 MHz
  a.sas = c->d_sas;
  a.gtab = c->d_gtab;
  a.tpair = c->d_tpair;
  a.nsas = c->cfg.max_sessions;              // unused entries are zero (mode 0): EINVAL
  __atomic_store_n(&c->door_ctl->stop, 0u, __ATOMIC_SEQ_CST);
  c->door_retiring = false;
  if (launch_gcm_door(a, c->door_wg, c->s_door)) return fail(c, ESPGPU_EIO, "door kernel launch failed");
  HIPCHK(c, hipEventRecord(c->ev_door, c->s_door));
  c->door_live = true;
  return 0;
}

// Relaunch the kernel if it exited (idle timeout) while jobs are outstanding.
int door_ensure(espgpu_ctx *c) {
  return door_exited(c) ? door_launch(c) : 0;
}

int door_setup(espgpu_ctx *c) {
  if (c->door_ctl) return 0;
  if (c->slots.size() > kDoorRing) return fail(c, ESPGPU_EINVAL, "door: more staging slots than ring entries (%u)", kDoorRing);
  HIPCHK(c, hipHostMalloc((void **)&c->door_ctl, sizeof(DoorCtl), hipHostMallocMapped | hipHostMallocCoherent));
  memset(c->door_ctl, 0, sizeof(DoorCtl));
  HIPCHK(c, hipHostGetDevicePointer((void **)&c->door_ctl_dev, c->door_ctl, 0));
  HIPCHK(c, hipMalloc(&c->d_door, sizeof(DoorDev)));
  HIPCHK(c, hipMemset(c->d_door, 0, sizeof(DoorDev)));
  HIPCHK(c, hipMalloc(&c->d_door_slots, c->slots.size() * sizeof(DoorSlot)));
  HIPCHK(c, hipStreamCreateWithFlags(&c->s_door, hipStreamNonBlocking));
  HIPCHK(c, hipEventCreateWithFlags(&c->ev_door, hipEventDisableTiming));
  const uint32_t cap = 3 * c->cfg.batch_records;     // xin + 2 xout spans per record
  for (size_t k = 0; k < c->slots.size(); ++k) {
    Slot &s = c->slots[k];
    if (s.xfer_cap < cap) {
      hipHostFree(s.h_xfer);
      s.h_xfer = nullptr;
      s.xfer_cap = 0;
      HIPCHK(c, hipHostMalloc((void **)&s.h_xfer, (size_t)cap * sizeof(XferSpan), hipHostMallocDefault));
      HIPCHK(c, hipHostGetDevicePointer((void **)&s.h_xfer_dev, s.h_xfer, 0));
      s.xfer_cap = cap;
    }
    HIPCHK(c, hipMalloc(&s.d_ej0, (size_t)c->cfg.batch_records * sizeof(uint4)));
    int e = door_write_slot(c, k);
    if (e) return e;
  }
  c->door_next = 0;
  return 0;
}

void door_free(espgpu_ctx *c) {
  door_stop(c);
  if (c->door_ctl) hipHostFree(c->door_ctl);
  hipFree(c->d_door);
  hipFree(c->d_door_slots);
  if (c->ev_door) hipEventDestroy(c->ev_door);
  if (c->s_door) hipStreamDestroy(c->s_door);
  c->door_ctl = c->door_ctl_dev = nullptr;
  c->d_door = nullptr;
  c->d_door_slots = nullptr;
  c->ev_door = nullptr;
  c->s_door = nullptr;
}

bool door_done(const espgpu_ctx *c, int64_t job) {
  const uint32_t j = (uint32_t)job;
  return __atomic_load_n(&c->door_ctl->done[j % kDoorRing], __ATOMIC_ACQUIRE) == j + 1;
}

// ---- GPU failure --------------------------------------------
// A launch or copy that cannot be queued, a completion query that returns an
// error, or a batch outstanding for deadline_ms is a GPU failure.  The ctx
// then launches nothing again, and every request it holds completes exactly
// once (crypto_done once per cryptop, crypto.c:1802-1804): with ESPGPU_EIO
// -- which the kernel-domain driver maps to EIO, a clean drop for
// esp_input_cb / esp_output_cb (esps_noxform, xform_esp.c:514-520) -- unless
// its batch is seen to complete after all (then with its real result).
// espgpu_health() reports the state: the F-Stack shim's probe then declines,
// so new SAs go to cryptosoft, and process() refuses at once.

// Wait, at most deadline_ms, for a stream's queued work; true if it drained
// (or the device reports an error: nothing of it runs any more).
bool stream_settle(espgpu_ctx *c, hipStream_t st) {
  if (!st) return true;
  const uint64_t t0 = now_ns();
  for (;;) {
    const hipError_t q = hipStreamQuery(st);
    if (q != hipErrorNotReady) return true;
    if (now_ns() - t0 > (uint64_t)c->deadline_ms * 1000000ull) return false;
    sched_yield();
  }
}

// A slot's requests complete with ESPGPU_EIO (their buffers untouched: results
// are copied back only for a batch that completed); the slot is free again.
void drop_slot(espgpu_ctx *c, Slot &s) {
  for (const Pending &pd : s.reqs) c->ready.push_back(espgpu_completion{pd.opaque, ESPGPU_EIO});
  c->stats.fail_eio += s.reqs.size();
  s.reqs.clear();
  s.segpool.clear();
  s.nrec = 0;
  s.bytes = 0;
  s.door_job = -1;
  s.stuck = false;
  s.state = SLOT_FREE;
}

// A batch about to be released as failed: work of it still queued may write
// the requests' host buffers (zero-copy results, the results' xfer kernel), so
// wait for its completion event, at most deadline_ms, first (as fail_launch
// does for a launch that failed part way).  A query error ends the wait: the
// device runs nothing of it any more.
void slot_settle(espgpu_ctx *c, Slot &s) {
  const uint64_t t0 = now_ns();
  while (hipEventQuery(s.done) == hipErrorNotReady) {
    if (now_ns() - t0 > (uint64_t)c->deadline_ms * 1000000ull) return;
    sched_yield();
  }
}

// Mark the ctx failed (once) and release what was never handed to the
// device: the filling slot and the host overflow.  In-flight batches are
// retired by poll / drain (slot_check).  Returns ESPGPU_EIO.
int ctx_fail(espgpu_ctx *c, const char *why) {
  if (!c->failed) {
    const std::string cause = c->err;
    c->failed = true;
    c->stats.gpu_fail++;
    c->err = std::string("GPU failure: ") + why + (cause.empty() ? "" : " (" + cause + ")");
    fprintf(stderr, "espgpu: %s; nothing more is launched, held requests complete with EIO\n", c->err.c_str());
    if (c->door_ctl) door_stop(c);               // (failed: asks the kernel to exit, never waits)
  }
  for (Slot &s : c->slots)
    if (s.state == SLOT_FILLING) drop_slot(c, s);
  Overflow &o = c->ovf;
  while (!o.empty()) {
    c->ready.push_back(espgpu_completion{o.front().pd.opaque, ESPGPU_EIO});
    c->stats.fail_eio++;
    o.pop();
  }
  return ESPGPU_EIO;
}

// Where an in-flight batch stands: 1 completed, 0 still running, -1 failed
// (its completion query returned an error, it outlived deadline_ms, or the ctx
// failed and the batch can no longer finish).  A doorbell job of a failed ctx
// is released only once the kernel has exited (a workgroup inside one of its
// chunks still writes results into host memory) or after the deadline; any
// other failed batch once its queued work has drained (slot_settle).
int slot_check(espgpu_ctx *c, Slot &s, uint64_t now) {
  const bool late = now > s.t_launch && now - s.t_launch > (uint64_t)c->deadline_ms * 1000000ull;
  if (s.door_job >= 0) {
    if (!s.stuck && door_done(c, s.door_job)) return 1;
    if (!c->failed && !late) return 0;
    if (!c->failed) ctx_fail(c, "doorbell job outstanding past deadline_ms");
    return (door_exited(c) || late) ? -1 : 0;
  }
  hipError_t q = s.stuck ? hipErrorNotReady : hipEventQuery(s.done);
  if (c->fault & ESPGPU_FAULT_QUERY) {
    c->fault &= ~(uint32_t)ESPGPU_FAULT_QUERY;
    q = hipErrorLaunchFailure;                   // injected: as a lost device reports it
  }
  if (q == hipSuccess) return 1;
  if (q != hipErrorNotReady) {
    if (!c->failed) {
      c->err = hipGetErrorString(q);
      ctx_fail(c, "batch completion query failed");
    }
    slot_settle(c, s);
    return -1;
  }
  if (!late) return 0;
  if (!c->failed) ctx_fail(c, "batch outstanding past deadline_ms");
  slot_settle(c, s);
  return -1;
}

// A slot whose launch failed part way: work already queued for it that
// writes host memory (a self-staging kernel, the results' xfer kernel or
// D2H copy) is waited for, boundedly, before its requests are released -- a
// released buffer must not be written afterwards.
int fail_launch(espgpu_ctx *c, Slot &s) {
  if (s.wq) stream_settle(c, s.wq);
  s.wq = nullptr;
  return ctx_fail(c, "batch launch failed");
}

// A slot's span list of at least `need` entries (the door's fixed layout
// keeps 3 x batch_records; a larger list moves the pinned buffer, so the
// door kernel is stopped first and the device slot table rewritten).
int xfer_reserve(espgpu_ctx *c, Slot &s, uint32_t need) {
  if (need <= s.xfer_cap) return 0;
  if (c->door_ctl) door_stop(c);
  hipHostFree(s.h_xfer);
  s.h_xfer = nullptr;
  s.xfer_cap = 0;
  const uint32_t cap = std::max(need, 256u) * 2;
  HIPCHK(c, hipHostMalloc((void **)&s.h_xfer, (size_t)cap * sizeof(XferSpan), hipHostMallocDefault));
  HIPCHK(c, hipHostGetDevicePointer((void **)&s.h_xfer_dev, s.h_xfer, 0));
  s.xfer_cap = cap;
  if (c->door_ctl) return door_write_slot(c, (size_t)(&s - c->slots.data()));
  return 0;
}

// Launch the crypto kernels for one batch of device-resident records.
// kinds: which kernels the batch needs (1 GCM, 2 ETA); the device-resident
// entry points do not know and pass both.
// The self-staging lists of a small single-session GCM process batch
// (GcmParams::xin / xout / hstat).
struct StageLists {
  const XferSpan *xin, *xout;
  uint8_t *hstat;
  const espgpu_desc *hdesc;
};

int run_batch(espgpu_ctx *c, uint8_t *d_arena, const espgpu_desc *d_desc, uint32_t n,
              uint8_t *d_status, uint8_t *d_out, uint32_t flags, int encrypt, hipStream_t st,
              uint32_t *d_trailer = nullptr, uint32_t kinds = 3, const StageLists *stage = nullptr,
              uint32_t out_stride = 0) {
  if (c->failed) return ESPGPU_EIO;
  if (n == 0) return 0;
  if (out_stride && c->n_eta > 0)
    return fail(c, ESPGPU_ENOTSUP, "packed output serves contexts with GCM sessions only");
  if (c->fault & ESPGPU_FAULT_LAUNCH) {
    c->fault &= ~(uint32_t)ESPGPU_FAULT_LAUNCH;
    return fail(c, ESPGPU_EIO, "injected launch failure");
  }
  door_retire(c);
  if (c->launched && st != c->last_st) HIPCHK(c, hipStreamWaitEvent(st, c->ev_last, 0));
  const uint32_t nsas = (uint32_t)c->sessions.size();
  GcmParams p{};
  p.arena = d_arena;
  p.out = encrypt ? d_arena : (d_out ? d_out : d_arena);
  p.desc = d_desc;
  p.n = n;
  p.sas = c->d_sas;
  p.gtab = c->d_gtab;
  p.tpair = c->d_tpair;
  p.status = d_status;
  p.nsas = nsas;
  p.queue = c->d_queue;
  p.trailer = encrypt ? nullptr : d_trailer;
  p.out_stride = out_stride;
  if (stage) {
    p.xin = stage->xin;
    p.xout = stage->xout;
    p.hstat = stage->hstat;
    p.hdesc = stage->hdesc;
  }
  if (!(flags & ESPGPU_BATCH_GROUPED)) {
    int e = ensure_plan(c, n);
    if (e) return e;
    // the key counts start at zero: plan_scatter zeroes them after use, so
    // only a fresh workspace (or one a failed launch left behind) needs it
    if (c->plan_dirty) {
      HIPCHK(c, hipMemsetAsync(c->d_work, 0, plan_workspace_words(c->cfg.max_sessions) * 4, st));
      c->plan_dirty = false;
    }
    if (launch_plan(d_desc, n, c->d_sas, nsas, c->cfg.max_sessions, c->d_work, c->d_order, c->d_chunks, c->d_nchunks,
                    c->max_chunks, st)) {
      c->plan_dirty = true;
      return fail(c, ESPGPU_EIO, "planner launch failed (%u sessions)", nsas);
    }
    p.order = c->d_order;
    p.chunks = c->d_chunks;
    p.nchunks = c->d_nchunks;
  }
  const int two_pass = (!encrypt && p.out == d_arena);
  // E_K(J0) scratch: the burst kernel (small batches of <= gcm_burst records,
  // out of place or encrypt; launch_gcm picks the kernel from it)
  const bool gsmall = c->gcm_lanes ? c->gcm_lanes == kGcmLanesSmall : n < kGcmSmallBatch;
  // (packed output: the fused kernel only)
  if ((kinds & 1) && !out_stride &&
      gsmall && !two_pass && n <= c->gcm_burst) {
    if (n > c->ej0_cap) {
      hipFree(c->d_ej0);
      c->d_ej0 = nullptr;
      c->ej0_cap = 0;
      HIPCHK(c, hipMalloc(&c->d_ej0, (size_t)n * sizeof(uint4)));
      c->ej0_cap = n;
    }
    p.ej0 = c->d_ej0;
  }
  // beside a running doorbell kernel (one workgroup per CU on door_wg CUs)
  // the other kernels take the remaining CUs: every workgroup of theirs must
  // run for the launch to finish
  int grid = c->cfg.grid ? (int)c->cfg.grid : 256;
  if (c->door_live && !door_exited(c)) grid = std::max(1, grid - c->door_wg);
  // A context without GCM sessions still launches the GCM kernel for the
  // records whose session is invalid (EINVAL; the planner chunks them with the
  // GCM records), but a few workgroups do: the others would only draw a
  // ticket past the end (cfg3: ~9 us -> ~3 us per batch)
  const int ggrid = c->n_gcm > 0 ? grid : std::min(grid, 16);
  if ((kinds & 1) && launch_gcm(p, encrypt, two_pass, ggrid, c->gcm_lanes, st))
    return fail(c, ESPGPU_EIO, "GCM kernel launch failed");
  if ((kinds & 2) && c->n_eta > 0) {
    EtaParams q{};
    q.arena = d_arena;
    q.out = p.out;
    q.desc = d_desc;
    q.order = p.order;
    q.chunks = p.chunks;
    q.nchunks = p.nchunks;
    q.queue = c->d_queue + kQueueRegionWords;
    q.trailer = p.trailer;
    q.n = n;
    q.sas = c->d_sas;
    q.tpair = c->d_tpair;
    q.dpair = c->d_dpair;
    q.isbox = c->d_isbox;
    q.status = d_status;
    q.nsas = nsas;
    const int ek = (c->n_cbc > 0 ? 1 : 0) | (c->n_ctr > 0 ? 2 : 0) | (c->n_wcbc > 0 ? 4 : 0) |
                   (c->n_wctr > 0 ? 8 : 0) | (c->n_whash > 0 ? 16 : 0);
    if (launch_eta(q, encrypt, ek, grid, st))
      return fail(c, ESPGPU_EIO, "ETA kernel launch failed");
  }
  HIPCHK(c, hipEventRecord(c->ev_last, st));
  c->last_st = st;
  c->launched = true;
  return 0;
}

}  // namespace

extern "C" {

int espgpu_abi_version(void) { return ESPGPU_ABI_VERSION; }

int espgpu_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : ESPGPU_ENODEV;
}

const char *espgpu_last_error(espgpu_ctx *c) { return c ? c->err.c_str() : "no context"; }

int espgpu_health(espgpu_ctx *c) {
  if (!c) return ESPGPU_EINVAL;
  return c->failed ? ESPGPU_EIO : ESPGPU_OK;
}

int espgpu_init(const espgpu_config *cfg_in, espgpu_ctx **out) {
  if (!out) return ESPGPU_EINVAL;
  *out = nullptr;
  espgpu_ctx *c = new espgpu_ctx();
  espgpu_config cfg{};
  if (cfg_in) cfg = *cfg_in;
  if (!cfg.max_sessions) cfg.max_sessions = 1024;
  if (!cfg.batch_records) cfg.batch_records = 65536;
  if (!cfg.batch_bytes) cfg.batch_bytes = 64u << 20;
  if (!cfg.nbatches) cfg.nbatches = 2;
  c->cfg = cfg;
  c->device = cfg.device;
  int rc = 0;
  do {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= cfg.device) {
      rc = fail(c, ESPGPU_ENODEV, "no HIP device %d (found %d)", cfg.device, ndev);
      break;
    }
    if (hipSetDevice(cfg.device) != hipSuccess) { rc = fail(c, ESPGPU_ENODEV, "hipSetDevice failed"); break; }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->s_in, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking) != hipSuccess) {
      rc = fail(c, ESPGPU_EIO, "stream");
      break;
    }
    for (int k = 0; k < 2; ++k) {
      hipEventCreateWithFlags(&c->e2e_in[k], hipEventDisableTiming);
      hipEventCreateWithFlags(&c->e2e_k[k], hipEventDisableTiming);
    }
    hipEventCreate(&c->ev0);
    hipEventCreate(&c->ev1);
    hipEventCreateWithFlags(&c->ev_last, hipEventDisableTiming);
    c->ready.reserve((size_t)cfg.batch_records * cfg.nbatches + 1024);
    if (hipMalloc(&c->d_sas, (size_t)cfg.max_sessions * sizeof(DevSA)) != hipSuccess ||
        hipMalloc(&c->d_gtab, (size_t)cfg.max_sessions * kGhTableBytes) != hipSuccess ||
        hipMalloc(&c->d_tpair, 256 * sizeof(uint2)) != hipSuccess ||
        hipMalloc(&c->d_dpair, 256 * sizeof(uint2)) != hipSuccess ||
        hipMalloc(&c->d_isbox, 256) != hipSuccess ||
        hipMalloc(&c->d_queue, 4 * kQueueRegionWords * 4) != hipSuccess) {
      rc = fail(c, ESPGPU_ENOMEM, "device SA table allocation failed");
      break;
    }
    hipMemset(c->d_sas, 0, (size_t)cfg.max_sessions * sizeof(DevSA));
    hipMemset(c->d_queue, 0, 4 * kQueueRegionWords * 4);
    const hc::Tables &t = hc::tables();
    uint2 tp[256], dp[256];
    for (int x = 0; x < 256; ++x) {
      tp[x] = make_uint2(t.te0[x], (t.te0[x] >> 8) | (t.te0[x] << 24));
      dp[x] = make_uint2(t.td0[x], (t.td0[x] >> 8) | (t.td0[x] << 24));
    }
    hipMemcpy(c->d_tpair, tp, sizeof tp, hipMemcpyHostToDevice);
    hipMemcpy(c->d_dpair, dp, sizeof dp, hipMemcpyHostToDevice);
    hipMemcpy(c->d_isbox, t.isbox, 256, hipMemcpyHostToDevice);
    c->slots.resize(cfg.nbatches);
    for (auto &s : c->slots)
      if ((rc = alloc_slot(c, s))) break;
  } while (0);
  if (rc) {
    fprintf(stderr, "espgpu_init: %s\n", c->err.c_str());
    espgpu_fini(c);
    return rc;
  }
  *out = c;
  return 0;
}

void espgpu_fini(espgpu_ctx *c) {
  if (!c) return;
  if (c->failed) {
    // nothing waits unboundedly on a failed device: work that may still run
    // on it (a hung kernel) keeps its memory, which is then leaked rather
    // than freed under it
    bool idle = true;
    const uint64_t t0 = now_ns();
    while (c->door_live && !door_exited(c)) {
      if (now_ns() - t0 > (uint64_t)c->deadline_ms * 1000000ull) { idle = false; break; }
      sched_yield();
    }
    for (hipStream_t st : {c->s_in, c->stream, c->s_out}) idle = stream_settle(c, st) && idle;
    for (auto &s : c->slots) idle = stream_settle(c, s.st) && idle;
    if (!idle) {
      fprintf(stderr, "espgpu_fini: device work of a failed context never finished; its memory is leaked\n");
      delete c;
      return;
    }
  }
  door_free(c);
  for (hipStream_t st : {c->s_in, c->stream, c->s_out})
    if (st) hipStreamSynchronize(st);
  for (auto &s : c->slots) free_slot(s);
  for (const HostRegion &r : c->regions)
    if (r.owned) hipHostUnregister((void *)r.base);
  hipFree(c->e2e_arena); hipFree(c->e2e_out); hipFree(c->e2e_status); hipFree(c->e2e_desc);
  for (int k = 0; k < 2; ++k) {
    if (c->e2e_in[k]) hipEventDestroy(c->e2e_in[k]);
    if (c->e2e_k[k]) hipEventDestroy(c->e2e_k[k]);
  }
  hipFree(c->d_sas); hipFree(c->d_gtab); hipFree(c->d_tpair); hipFree(c->d_dpair); hipFree(c->d_isbox);
  hipFree(c->d_queue);
  hipFree(c->d_ej0);
  hipFree(c->d_work); hipFree(c->d_order); hipFree(c->d_chunks); hipFree(c->d_nchunks);
  if (c->ev0) hipEventDestroy(c->ev0);
  if (c->ev1) hipEventDestroy(c->ev1);
  if (c->ev_last) hipEventDestroy(c->ev_last);
  for (hipStream_t st : {c->s_in, c->stream, c->s_out})
    if (st) hipStreamDestroy(st);
  delete c;
}

// swcr_probesession + check_csp restricted to the ESP ciphers this engine serves.
int espgpu_probesession(const espgpu_session_params *csp) {
  if (!csp) return ESPGPU_EINVAL;
  const int supported_flags = ESPGPU_CSP_F_SEPARATE_AAD | ESPGPU_CSP_F_ESN;
  if (csp->csp_flags & ~supported_flags) return ESPGPU_EINVAL;
  if (csp->csp_ivlen < 0 || csp->csp_cipher_klen < 0 || csp->csp_auth_klen < 0 || csp->csp_auth_mlen < 0)
    return ESPGPU_EINVAL;
  const int k = csp->csp_cipher_klen;
  const bool aes_klen = (k == 16 || k == 24 || k == 32);
  switch (csp->csp_mode) {
    case ESPGPU_CSP_MODE_AEAD:
      if (csp->csp_cipher_alg != ESPGPU_CRYPTO_AES_NIST_GCM_16 || !aes_klen) return ESPGPU_EINVAL;
      if (csp->csp_ivlen != 12) return ESPGPU_EINVAL;                 // cryptosoft.c:1093
      if (csp->csp_auth_alg != 0 || csp->csp_auth_klen != 0) return ESPGPU_EINVAL;
      // ICVs of 8/12/16 bytes (RFC 4106 s3.3; 0 = 16); other truncations,
      // which ESP never sets up, are left to cryptosoft (probe ESPGPU_EINVAL)
      if (csp->csp_auth_mlen != 0 && csp->csp_auth_mlen != 8 && csp->csp_auth_mlen != 12 &&
          csp->csp_auth_mlen != 16)
        return ESPGPU_EINVAL;
      if (csp->csp_flags & ESPGPU_CSP_F_ESN) return ESPGPU_EINVAL;    // ESN for GCM = SEPARATE_AAD
      return ESPGPU_PROBE_HARDWARE;
    case ESPGPU_CSP_MODE_CIPHER:
      // ESP with encryption and no auth (esp_init :230-231): AES-CBC or
      // AES-ICM (csp_ivlen = the enc_xform's 16), or ESP-NULL (no key, no
      // IV: swcr_null); swcr_probesession :1257-1266 / swcr_cipher_supported
      // :1228-1239.  No auth fields; esp_init sets no flags for it.
      if (csp->csp_auth_alg != 0 || csp->csp_auth_klen != 0 || csp->csp_auth_mlen != 0) return ESPGPU_EINVAL;
      if (csp->csp_flags) return ESPGPU_EINVAL;
      if (csp->csp_cipher_alg == ESPGPU_CRYPTO_NULL_CBC) return csp->csp_cipher_klen == 0 ? ESPGPU_PROBE_HARDWARE : ESPGPU_EINVAL;
      if ((csp->csp_cipher_alg != ESPGPU_CRYPTO_AES_CBC && csp->csp_cipher_alg != ESPGPU_CRYPTO_AES_ICM) ||
          !aes_klen || csp->csp_ivlen != 16)
        return ESPGPU_EINVAL;
      return ESPGPU_PROBE_HARDWARE;
    case ESPGPU_CSP_MODE_ETA: {
      // AES-CBC or AES-ICM (CTR; csp_ivlen = the enc_xform's 16, the nonce
      // rides in crp_iv), or ESP-NULL (CRYPTO_NULL_CBC: no key; cryptosoft
      // degrades the session to the digest, cryptosoft.c:1394-1398), with
      // HMAC-SHA1 or HMAC-SHA2-256/384/512 (esp_init :225-241)
      if (csp->csp_cipher_alg == ESPGPU_CRYPTO_NULL_CBC) {
        if (csp->csp_cipher_klen != 0) return ESPGPU_EINVAL;
      } else if ((csp->csp_cipher_alg != ESPGPU_CRYPTO_AES_CBC && csp->csp_cipher_alg != ESPGPU_CRYPTO_AES_ICM) ||
                 !aes_klen || csp->csp_ivlen != 16) {
        return ESPGPU_EINVAL;
      }
      int hashlen = 0;
      switch (csp->csp_auth_alg) {                                 // xform_sha1.c, xform_sha2.c
        case ESPGPU_CRYPTO_SHA1_HMAC: hashlen = 20; break;
        case ESPGPU_CRYPTO_SHA2_256_HMAC: hashlen = 32; break;
        case ESPGPU_CRYPTO_SHA2_384_HMAC: hashlen = 48; break;
        case ESPGPU_CRYPTO_SHA2_512_HMAC: hashlen = 64; break;
      }
      if (!hashlen || csp->csp_auth_klen <= 0) return ESPGPU_EINVAL;
      if (csp->csp_auth_mlen > hashlen || (csp->csp_auth_mlen & 3)) return ESPGPU_EINVAL;
      if (csp->csp_flags & ESPGPU_CSP_F_SEPARATE_AAD) return ESPGPU_EINVAL;
      return ESPGPU_PROBE_HARDWARE;
    }
    default:
      return ESPGPU_EINVAL;
  }
}

int espgpu_newsession(espgpu_ctx *c, const espgpu_session_params *csp, int32_t *sid_out) {
  if (!c || !csp || !sid_out) return ESPGPU_EINVAL;
  if (c->failed) return ESPGPU_EIO;                  // (espgpu_last_error keeps the cause)
  int pr = espgpu_probesession(csp);
  if (pr >= 0) return fail(c, ESPGPU_EINVAL, "session parameters not supported");
  const bool null_cipher = csp->csp_cipher_alg == ESPGPU_CRYPTO_NULL_CBC;
  if (!csp->csp_cipher_key && !null_cipher)
    return fail(c, ESPGPU_EINVAL, "per-request keys are not supported; session key required");
  int slot = -1;
  for (size_t i = 0; i < c->sessions.size(); ++i)
    if (!c->sessions[i].used) { slot = (int)i; break; }
  if (slot < 0) {
    if (c->sessions.size() >= c->cfg.max_sessions) return fail(c, ESPGPU_ENOMEM, "SA table full (%u)", c->cfg.max_sessions);
    slot = (int)c->sessions.size();
    c->sessions.emplace_back();
    c->h_sas.emplace_back();
  }
  DevSA sa;
  memset(&sa, 0, sizeof sa);
  const uint8_t *key = (const uint8_t *)csp->csp_cipher_key;
  uint32_t rk[60];
  const int nr = null_cipher ? 0 : hc::aes_expand_enc(key, csp->csp_cipher_klen, rk);
  sa.nr = (uint32_t)nr;
  // CSP_MODE_CIPHER sessions run in the ETA kernels (aalg 0: no MAC pass)
  sa.mode = (uint32_t)(csp->csp_mode == ESPGPU_CSP_MODE_CIPHER ? ESPGPU_CSP_MODE_ETA : csp->csp_mode);
  sa.flags = (uint32_t)csp->csp_flags;
  if (csp->csp_mode == ESPGPU_CSP_MODE_AEAD) {
    sa.mlen = csp->csp_auth_mlen ? (uint32_t)csp->csp_auth_mlen : 16;
    // kernel form: raw first round, ror16 middle rounds, byte-swapped last round
    for (int i = 0; i < 4; ++i) sa.rk[i] = rk[i];
    for (int i = 4; i < 4 * nr; ++i) sa.rk[i] = ror16(rk[i]);
    for (int i = 0; i < 4; ++i) sa.rk[4 * nr + i] = bswap(rk[4 * nr + i]);
    // bitsliced ctr pass (aes_bs.h): K0, then K_r ^ 0x63..63 (the S-box
    // circuit's affine constant), little-endian words
    for (int i = 0; i < 4 * (nr + 1); ++i) sa.dk[i] = bswap(rk[i]) ^ (i >= 4 ? 0x63636363u : 0u);
    uint8_t zero[16] = {0}, h[16];
    hc::aes_encrypt_block(rk, nr, zero, h);       // H = E_K(0^128), gmac.c:56-60
    std::vector<uint8_t> tabs(kGhTableBytes);
    hc::ghash_tables(h, tabs.data());
    HIPCHK(c, hipMemcpy(c->d_gtab + (size_t)slot * kGhTableBytes, tabs.data(), kGhTableBytes, hipMemcpyHostToDevice));
  } else {
    const bool auth = csp->csp_mode == ESPGPU_CSP_MODE_ETA;
    const int aalg = auth ? csp->csp_auth_alg : 0;
    const bool sha256 = aalg == ESPGPU_CRYPTO_SHA2_256_HMAC;
    const bool wide = aalg == ESPGPU_CRYPTO_SHA2_384_HMAC || aalg == ESPGPU_CRYPTO_SHA2_512_HMAC;
    sa.calg = (uint32_t)csp->csp_cipher_alg;
    sa.aalg = (uint32_t)aalg;
    // mlen 0 = the whole hash (swcr_setup_auth, cryptosoft.c:1013-1018); no
    // ICV without auth
    const uint32_t hashlen = sha256 ? 32u : aalg == ESPGPU_CRYPTO_SHA2_384_HMAC ? 48u
                           : aalg == ESPGPU_CRYPTO_SHA2_512_HMAC ? 64u : 20u;
    sa.mlen = !auth ? 0u : csp->csp_auth_mlen ? (uint32_t)csp->csp_auth_mlen : hashlen;
    if (!null_cipher) {
      for (int i = 0; i < 4 * (nr + 1); ++i) sa.rk[i] = rk[i];
      uint32_t dk[60];
      hc::aes_expand_dec(key, csp->csp_cipher_klen, dk);
      for (int i = 0; i < 4 * (nr + 1); ++i) sa.dk[i] = dk[i];
    }
    const uint8_t *ak = (const uint8_t *)csp->csp_auth_key;
    if (!auth) {
    } else if (wide) {
      const bool is384 = aalg == ESPGPU_CRYPTO_SHA2_384_HMAC;
      hc::hmac_sha512_pad_state(ak, csp->csp_auth_klen, 0x36, is384, sa.ipad);
      hc::hmac_sha512_pad_state(ak, csp->csp_auth_klen, 0x5c, is384, sa.opad);
    } else if (sha256) {
      hc::hmac_sha256_pad_state(ak, csp->csp_auth_klen, 0x36, sa.ipad);
      hc::hmac_sha256_pad_state(ak, csp->csp_auth_klen, 0x5c, sa.opad);
    } else {
      hc::hmac_sha1_pad_state(ak, csp->csp_auth_klen, 0x36, sa.ipad);
      hc::hmac_sha1_pad_state(ak, csp->csp_auth_klen, 0x5c, sa.opad);
    }
  }
  HIPCHK(c, hipMemcpy(c->d_sas + slot, &sa, sizeof sa, hipMemcpyHostToDevice));
  Session &s = c->sessions[slot];
  s.used = true;
  s.mode = csp->csp_mode;
  s.flags = csp->csp_flags;
  s.mlen = (int)sa.mlen;
  s.klen = csp->csp_cipher_klen;
  const bool eta_kind = csp->csp_mode != ESPGPU_CSP_MODE_AEAD;
  s.ctr = eta_kind && csp->csp_cipher_alg == ESPGPU_CRYPTO_AES_ICM;
  s.null = eta_kind && null_cipher;
  s.whash = eta_kind && (sa.aalg == ESPGPU_CRYPTO_SHA2_384_HMAC || sa.aalg == ESPGPU_CRYPTO_SHA2_512_HMAC);
  s.wide = s.whash || (eta_kind && (sa.aalg == 0 || null_cipher));
  if (eta_kind) {
    c->n_eta++;
    eta_count(c, s)++;
    c->n_whash += s.whash ? 1 : 0;
  } else {
    c->n_gcm++;
  }
  c->h_sas[slot] = sa;
  *sid_out = slot;
  return 0;
}

int espgpu_session_room(espgpu_ctx *c) {
  if (!c) return ESPGPU_EINVAL;
  size_t room = c->cfg.max_sessions - c->sessions.size();
  for (const Session &s : c->sessions) room += s.used ? 0 : 1;
  return (int)std::min<size_t>(room, INT32_MAX);
}

void espgpu_freesession(espgpu_ctx *c, int32_t sid) {
  if (!c || sid < 0 || (size_t)sid >= c->sessions.size() || !c->sessions[sid].used) return;
  if (!c->failed) {
    // Requests already staged were accepted under this key: launch them now
    // (and the overflow behind them), then wait, so neither they nor flushed
    // batches see the slot reused.
    // (doorbell jobs have no stream to wait on: drain them)
    if (c->ovf.empty() && !c->door_ctl) espgpu_flush(c);
    else espgpu_drain(c);
  }
  if (!c->failed) {
    // the doorbell kernel keeps its current session's state (H^8 table in LDS);
    // stopped before the stream syncs, which could otherwise wait behind it
    // on a shared hardware queue
    door_stop(c);
    hipStreamSynchronize(c->stream);
    hipStreamSynchronize(c->s_out);
    for (auto &sl : c->slots) hipStreamSynchronize(sl.st);
    // and the ctx's last launch on any stream: a device-resident batch on the
    // caller's stream may still be reading this slot's keys
    if (c->launched) hipEventSynchronize(c->ev_last);
  }
  const Session &fs = c->sessions[sid];
  if (fs.mode != ESPGPU_CSP_MODE_AEAD) {
    c->n_eta--;
    eta_count(c, fs)--;
    c->n_whash -= fs.whash ? 1 : 0;
  } else {
    c->n_gcm--;
  }
  c->sessions[sid] = Session();
  DevSA z;
  memset(&z, 0, sizeof z);
  if (!c->failed) hipMemcpy(c->d_sas + sid, &z, sizeof z, hipMemcpyHostToDevice);
}

// Validate that a request has the shape esp_input / esp_output build
// (xform_esp.c:364-461, 820-900) and stage it as an ESP wire record.
int espgpu_process(espgpu_ctx *c, const espgpu_req *r, int hint) {
  (void)hint;
  if (!c || !r) return ESPGPU_EINVAL;
  if (c->failed) {
    // never ERESTART (nothing would retry it into a working slot) nor EAGAIN:
    // the caller completes it at once (ff_gpucrypto.c)
    c->stats.fail_eio++;
    return ESPGPU_EIO;
  }
  const int op = (r->crp_op & ESPGPU_CRYPTO_OP_ENCRYPT) ? 1 : 0;
  auto reject = [&](int etype) {
    c->ready.push_back(espgpu_completion{r->opaque, etype});
    if (etype == ESPGPU_EINVAL) c->stats.einval++;
    return 0;
  };
  const int sid = r->session;
  if (sid < 0 || (size_t)sid >= c->sessions.size() || !c->sessions[sid].used) return reject(ESPGPU_EINVAL);
  const Session &ses = c->sessions[sid];
  size_t total = 0;
  for (int i = 0; i < r->nsegs; ++i) total += r->segs[i].len;
  const bool gcm = ses.mode == ESPGPU_CSP_MODE_AEAD, cipher_only = ses.mode == ESPGPU_CSP_MODE_CIPHER;
  // ICV bytes in the record: the session's (possibly truncated) mlen, 16/12/8
  // for GCM (cryptosoft.c:1112-1117), 12 or 20 for HMAC-SHA1, 16 for
  // HMAC-SHA2-256-128, none without auth.  IV: 8 for GCM / CTR, none for
  // ESP-NULL (ivsize 0), else 16.
  const int ivlen = (gcm || ses.ctr) ? 8 : ses.null ? 0 : 16, hlen = 8 + ivlen, alen = ses.mlen;
  const int plen = r->crp_payload_length;
  int aad_start = cipher_only ? r->crp_payload_start - hlen : r->crp_aad_start;
  // ESP shape checks
  if (plen <= 0 || r->crp_payload_start < hlen ||
      (size_t)(r->crp_payload_start + plen + alen) > total ||
      (alen && (size_t)(r->crp_digest_start + alen) > total))
    return reject(ESPGPU_EINVAL);
  if (cipher_only && (r->crp_aad || r->crp_aad_length != 0 || (r->crp_op & ESPGPU_CRYPTO_OP_VERIFY_DIGEST)))
    return reject(ESPGPU_EINVAL);
  uint8_t hdr[8];
  uint32_t esn_hi = 0, salt = 0;
  if (gcm) {
    if (!(r->crp_flags & ESPGPU_CRYPTO_F_IV_SEPARATE)) return reject(ESPGPU_EINVAL);   // cryptosoft.c:496
    if (r->crp_aad) {
      if (!(ses.flags & ESPGPU_CSP_F_SEPARATE_AAD) || r->crp_aad_length != 12) return reject(ESPGPU_EINVAL);
      const uint8_t *a = (const uint8_t *)r->crp_aad;
      memcpy(hdr, a, 4);
      memcpy(hdr + 4, a + 8, 4);
      esn_hi = be32(a + 4);
      aad_start = r->crp_payload_start - hlen;   // header bytes in the buffer (unused by the cipher)
    } else {
      if (r->crp_aad_length != 8 || (ses.flags & ESPGPU_CSP_F_SEPARATE_AAD)) return reject(ESPGPU_EINVAL);
      if (r->crp_payload_start != aad_start + hlen) return reject(ESPGPU_EINVAL);
      if (!seg_copy_out(r->segs, (uint32_t)r->nsegs, (uint32_t)aad_start, 8, hdr)) return reject(ESPGPU_EINVAL);
    }
    salt = le32(r->crp_iv);
  } else if (ses.ctr) {
    // AES-CTR: crp_iv = nonce || explicit IV || be32(1) (xform_esp.c:453-458),
    // and the explicit IV is the record's; the kernel rebuilds the counter
    // blocks from the descriptor's salt (the nonce) and the record
    if (!(r->crp_flags & ESPGPU_CRYPTO_F_IV_SEPARATE) || r->crp_aad ||
        (!cipher_only && r->crp_aad_length != hlen) || r->crp_payload_start != aad_start + hlen ||
        be32(r->crp_iv + 12) != 1u)
      return reject(ESPGPU_EINVAL);
    uint8_t ivb[8];
    if (!seg_copy_out(r->segs, (uint32_t)r->nsegs, (uint32_t)(aad_start + 8), 8, ivb) ||
        memcmp(ivb, r->crp_iv + 4, 8) != 0)
      return reject(ESPGPU_EINVAL);
    salt = le32(r->crp_iv);
    if (ses.flags & ESPGPU_CSP_F_ESN) esn_hi = be32(r->crp_esn);
  } else if (ses.null) {
    // ESP-NULL: no IV (crp_iv_start unset, xform_esp.c:459-461), payload a
    // multiple of the null blocksize 4 (:316-324)
    if (r->crp_aad || (!cipher_only && r->crp_aad_length != hlen) || r->crp_payload_start != aad_start + hlen ||
        (plen & 3))
      return reject(ESPGPU_EINVAL);
    if (ses.flags & ESPGPU_CSP_F_ESN) esn_hi = be32(r->crp_esn);
  } else {
    if (r->crp_aad || (!cipher_only && r->crp_aad_length != hlen) || r->crp_iv_start != aad_start + 8 ||
        r->crp_payload_start != aad_start + hlen || (plen & 15))
      return reject(ESPGPU_EINVAL);
    if (ses.flags & ESPGPU_CSP_F_ESN) esn_hi = be32(r->crp_esn);
  }
  if (alen && r->crp_digest_start != r->crp_payload_start + plen) return reject(ESPGPU_EINVAL);
  const uint32_t rlen = (uint32_t)(hlen + plen + alen);
  if (rlen > 65535 || (rlen & 3) || rlen + 16 > c->cfg.batch_bytes) return reject(ESPGPU_EINVAL);
  // Zero-copy when the whole record lies in one segment of registered memory
  // with the layout the kernels read (the staged path takes a GCM record's
  // header and IV from crp_aad / crp_iv: they must equal the buffer's).
  const uint32_t rec_start = (uint32_t)(r->crp_payload_start - hlen);
  uint64_t zc = 0;
  if (!c->regions.empty()) {
    const uint8_t *rp = seg_span(r->segs, (uint32_t)r->nsegs, rec_start, rlen);
    if (rp && (!gcm || (memcmp(rp, hdr, 8) == 0 && memcmp(rp + 8, r->crp_iv + 4, 8) == 0)))
      zc = region_dev(c, rp, rlen);
  }
  // the record bytes as the kernels read them: SPI | SN | IV | payload | ICV
  auto gather = [&](uint8_t *dst) {
    if (gcm) {
      memcpy(dst, hdr, 8);
      memcpy(dst + 8, r->crp_iv + 4, 8);
      return seg_copy_out(r->segs, (uint32_t)r->nsegs, (uint32_t)r->crp_payload_start, (uint32_t)(plen + alen),
                          dst + hlen);
    }
    return seg_copy_out(r->segs, (uint32_t)r->nsegs, (uint32_t)aad_start, rlen, dst);
  };
  Pending pd;
  pd.opaque = r->opaque;
  pd.etype_pre = -1;
  pd.rec = 0;
  pd.stage_off = 0;
  pd.stage_len = rlen;
  pd.nsegs = (uint32_t)r->nsegs;
  pd.seg0 = 0;
  pd.zc = zc;
  // results: payload (+ digest when encrypting) go back to the request buffer
  pd.nspan = 1;
  pd.span[0] = {(uint32_t)r->crp_payload_start, (uint32_t)hlen, (uint32_t)plen};
  if (op == 1 && alen) {
    pd.nspan = 2;
    pd.span[1] = {(uint32_t)r->crp_digest_start, (uint32_t)(hlen + plen), (uint32_t)ses.mlen};
  }
  espgpu_desc d;
  d.off4 = 0;
  d.len = (uint16_t)rlen;
  d.sa = (uint16_t)sid;
  d.esn_hi = esn_hi;
  d.salt = salt;
  const uint8_t kind = gcm ? 1 : 2;
  // Where it goes: the filling slot; the overflow when the slots are all in
  // flight (or the overflow already holds requests: arrival order is kept);
  // else ERESTART.
  Slot *s = &c->slots[c->cur];
  bool to_ovf = !c->ovf.empty();
  if (!to_ovf) {
    if (slot_full(c, *s, op, rlen)) {
      int e = espgpu_flush(c);
      if (e) {
        if (c->failed) c->stats.fail_eio++;     // (this request: refused, completed by the caller)
        return e;
      }
      s = &c->slots[c->cur];
    }
    if (s->state == SLOT_INFLIGHT) {
      if (!c->ovf_cap) { c->stats.erestart++; return ESPGPU_ERESTART; }
      to_ovf = true;
    }
  }
  if (to_ovf) {
    // fixed rings reserved at set_tuning: nothing here allocates or moves
    const uint64_t t_in = now_ns();
    Overflow &o = c->ovf;
    const size_t blen = zc ? 0 : ((rlen + 15) & ~15u);
    if (o.count == o.ecap) { c->stats.erestart++; return ESPGPU_ERESTART; }
    const auto bm = o.bytes.mark();
    const auto sm = o.segpool.mark();
    const size_t boff = o.bytes.alloc(blen), soff = o.segpool.alloc((size_t)r->nsegs);
    if (boff == SIZE_MAX || soff == SIZE_MAX) {
      o.bytes.undo(bm);
      o.segpool.undo(sm);
      c->stats.erestart++;
      return ESPGPU_ERESTART;
    }
    pd.stage_off = (uint32_t)boff;
    if (!zc && !gather(o.bytes.buf.get() + boff)) {
      o.bytes.undo(bm);
      o.segpool.undo(sm);
      return reject(ESPGPU_EINVAL);
    }
    pd.seg0 = (uint32_t)soff;
    if (r->nsegs) memcpy(o.segpool.buf.get() + soff, r->segs, (size_t)r->nsegs * sizeof(espgpu_seg));
    o.ent[(o.head + o.count) % o.ecap] = OvfEntry{pd, d, sid, (uint8_t)op, kind};
    o.count++;
    o.live_bytes += blen;
    o.peak_bytes = std::max(o.peak_bytes, o.live_bytes);
    c->stats.overflow++;
    c->stats.ovf_process_ns_max = std::max(c->stats.ovf_process_ns_max, now_ns() - t_in);
    return 0;
  }
  if (!zc && !gather(s->h_arena + s->bytes)) return reject(ESPGPU_EINVAL);
  slot_commit(*s, pd, d, r->segs, sid, op, kind);
  return 0;
}

// Launch one filled slot: its staging region and zero-copy records in, the
// crypto kernels, the results out; then the next slot becomes current.
static int launch_slot(espgpu_ctx *c, Slot &s) {
  if (s.state != SLOT_FILLING || s.nrec == 0) return 0;
  s.wq = nullptr;
  if (c->fault & ESPGPU_FAULT_LAUNCH) {
    c->fault &= ~(uint32_t)ESPGPU_FAULT_LAUNCH;
    return fail(c, ESPGPU_EIO, "injected launch failure");
  }
  if (c->fault & ESPGPU_FAULT_STUCK) {            // its completion will never be seen
    c->fault &= ~(uint32_t)ESPGPU_FAULT_STUCK;
    s.stuck = true;
  }
  // [records][16 B slack][descriptors][status]: one H2D on s_in -> kernels on
  // the compute stream -> one D2H on s_out, chained by events, so consecutive
  // batches overlap their copies with each other's kernels.
  s.desc_off = s.bytes + 16;
  s.stat_off = s.desc_off + s.nrec * (uint32_t)sizeof(espgpu_desc);
  memset(s.h_arena + s.bytes, 0, 16);
  memcpy(s.h_arena + s.desc_off, s.h_desc, s.nrec * sizeof(espgpu_desc));
  // A small batch (an RX burst) runs in order on its slot's own stream:
  // cross-stream event hand-offs cost more latency than the copies; the next
  // slot's burst overlaps on the other slot's stream (kernels stay ordered
  // through run_batch's last-launch event).  Its staging region moves by the
  // xfer kernel (set_tuning "xfer", default) or hipMemcpyAsync.  Large
  // batches use the three ctx streams so batch k+1's H2D overlaps batch k's
  // kernels and batch k-1's D2H.  Zero-copy records move by the xfer kernel
  // on the compute stream either way.
  const bool small = s.stat_off <= kSmallBatchBytes;
  const bool kcopy = small && c->xfer_small;
  hipStream_t s_k = small ? s.st : c->stream;
  hipStream_t s_in = small ? s.st : c->s_in, s_out = small ? s.st : c->s_out;
  uint8_t *dres = s.op ? s.d_arena : s.d_out;      // records out: in place (encrypt) or d_out
  // A small batch of one GCM session stages its own records: the kernel's
  // workgroups copy each chunk's records in from the host (pinned staging or
  // registered memory) and the results back, reading the descriptors and
  // writing the statuses through the host mapping -- one launch per burst
  // instead of copy, kernel, copy (set_tuning "stage_fused"; the small-batch
  // GCM kernel, so not with gcm_lanes 4 forced)
  const bool one_gcm = !s.mixed && s.kinds == 1 && c->gcm_lanes != kGcmLanesPerRec;
  // Doorbell path (set_tuning "door"): a single-session GCM batch of up to
  // gcm_burst records is published to the persistent kernel -- descriptors
  // and span lists at the slot's fixed door offsets, then one 16-byte job in
  // the ring -- with no HIP call at all; poll() sees done[] in host memory.
  if (c->door_wg && one_gcm && s.nrec <= c->gcm_burst) {
    int e = door_setup(c);
    if (e) return e;
    s.desc_off = door_desc_off(c);
    s.stat_off = door_stat_off(c);
    memcpy(s.h_arena + s.desc_off, s.h_desc, s.nrec * sizeof(espgpu_desc));
    const uint64_t ha = (uint64_t)(uintptr_t)s.h_arena_dev, da = (uint64_t)(uintptr_t)s.d_arena;
    const uint64_t dr = (uint64_t)(uintptr_t)dres;
    XferSpan *xin = s.h_xfer, *xout = s.h_xfer + c->cfg.batch_records;
    for (const Pending &pd : s.reqs) {
      xin[pd.rec] = XferSpan{pd.zc ? pd.zc : ha + pd.stage_off, da + pd.stage_off, pd.stage_len, pd.rec};
      for (int q = 0; q < 2; ++q) {
        XferSpan &o = xout[2 * pd.rec + q];
        if (q < pd.nspan) {
          const Pending::Span &sp = pd.span[q];
          o = XferSpan{dr + pd.stage_off + sp.stage_from,
                       pd.zc ? pd.zc + sp.stage_from : ha + pd.stage_off + sp.stage_from, sp.n, pd.rec};
        } else {
          o = XferSpan{0, 0, 0, pd.rec};
        }
      }
    }
    // A kernel asked to retire (launched work went by) may still be running.
    // The request stands while that launched work is outstanding: the kernel
    // then serves the jobs published meanwhile and exits, so work queued
    // behind it on a shared hardware queue does not wait for door_idle_us.
    // Once the launched work is done the request is cancelled before the job
    // is visible.  A kernel that exited (the request, or an idle timeout since
    // the last job) is relaunched, which clears it.  All before the ring entry
    // is written, so a failed relaunch leaves nothing published.
    const uint64_t t_pub = now_ns();
    const bool was_retiring = c->door_retiring;
    if (was_retiring && launched_idle(c)) {
      __atomic_store_n(&c->door_ctl->stop, 0u, __ATOMIC_SEQ_CST);
      c->door_retiring = false;
    }
    if (!c->door_live || t_pub - c->door_last_pub > (uint64_t)c->door_idle_us * 500u ||
        (was_retiring && door_exited(c))) {
      e = door_ensure(c);
      if (e) return e;
    }
    const uint32_t j = c->door_next++;
    DoorJob &jb = c->door_ctl->ring[j % kDoorRing];
    const uint32_t so = (uint32_t)(&s - c->slots.data()) | ((uint32_t)s.op << 16);
    jb.n = s.nrec;
    jb.slot_op = so;
    jb.chk = s.nrec ^ so ^ (j + 1) ^ kDoorChk;
    __atomic_store_n(&jb.seq, j + 1, __ATOMIC_RELEASE);
    s.door_job = j;
    s.door_t0 = t_pub;
    c->door_last_pub = t_pub;
    s.timed = false;
    s.t_launch = now_ns();               // (the deadline counts from here: launch calls may load code)
    s.state = SLOT_INFLIGHT;
    c->stats.batches++;
    c->stats.door++;
    c->stats.zerocopy += s.nrec - s.nstaged;
    c->cur = (c->cur + 1) % (int)c->slots.size();
    return 0;
  }
  door_retire(c);                                  // launched work from here on
  if (small && c->stage_fused && one_gcm) {
    int e = xfer_reserve(c, s, 3 * s.nrec);
    if (e) return e;
    const uint64_t ha = (uint64_t)(uintptr_t)s.h_arena_dev, da = (uint64_t)(uintptr_t)s.d_arena;
    const uint64_t dr = (uint64_t)(uintptr_t)dres;
    XferSpan *xin = s.h_xfer, *xout = s.h_xfer + s.nrec;
    for (const Pending &pd : s.reqs) {
      xin[pd.rec] = XferSpan{pd.zc ? pd.zc : ha + pd.stage_off, da + pd.stage_off, pd.stage_len, pd.rec};
      for (int q = 0; q < 2; ++q) {
        XferSpan &o = xout[2 * pd.rec + q];
        if (q < pd.nspan) {
          const Pending::Span &sp = pd.span[q];
          o = XferSpan{dr + pd.stage_off + sp.stage_from,
                       pd.zc ? pd.zc + sp.stage_from : ha + pd.stage_off + sp.stage_from, sp.n, pd.rec};
        } else {
          o = XferSpan{0, 0, 0, pd.rec};
        }
      }
    }
    const StageLists stg{s.h_xfer_dev, s.h_xfer_dev + s.nrec, s.h_arena_dev + s.stat_off,
                         reinterpret_cast<const espgpu_desc *>(s.h_arena_dev + s.desc_off)};
    s.timed = GPU_TIME_SMALL;
    if (s.timed) hipEventRecord(s.k0, s_k);
    s.wq = s_k;                                    // the kernel writes results to host memory
    e = run_batch(c, s.d_arena, reinterpret_cast<const espgpu_desc *>(s.d_arena + s.desc_off), s.nrec,
                  dres + s.stat_off, s.op ? nullptr : s.d_out, (uint32_t)ESPGPU_BATCH_GROUPED, s.op, s_k,
                  nullptr, 1u, &stg);
    if (e) return e;
    if (s.timed) hipEventRecord(s.k1, s_k);
    HIPCHK(c, hipEventRecord(s.done, s_k));
    s.t_launch = now_ns();               // (the deadline counts from here: launch calls may load code)
    s.state = SLOT_INFLIGHT;
    c->stats.batches++;
    c->stats.zerocopy += s.nrec - s.nstaged;
    c->cur = (c->cur + 1) % (int)c->slots.size();
    return 0;
  }
  // region the copies move: all of it, or without records if every one is zero-copy
  const uint32_t in_lo = s.nstaged ? 0 : s.desc_off, out_lo = s.nstaged ? 0 : s.stat_off;
  const uint32_t out_hi = s.stat_off + s.nrec;
  auto pieces = [](uint32_t n) { return (n + kXferPiece - 1) / kXferPiece; };
  uint32_t nin = 0, nout = 0;
  for (const Pending &pd : s.reqs) {
    if (pd.zc) {
      nin += pieces(pd.stage_len);
      for (int k = 0; k < pd.nspan; ++k) nout += pieces(pd.span[k].n);
    } else if (kcopy) {
      nin += pieces(pd.stage_len);
      nout += pieces(pd.stage_len);
    }
  }
  if (kcopy) {
    nin += pieces(s.stat_off - s.desc_off);
    nout += pieces(s.nrec);
  }
  {
    int e = xfer_reserve(c, s, nin + nout);
    if (e) return e;
  }
  uint32_t k = 0;
  auto add = [&](uint64_t src, uint64_t dst, uint32_t n, uint32_t rec) {
    for (uint32_t o = 0; o < n; o += kXferPiece)
      s.h_xfer[k++] = XferSpan{src + o, dst + o, std::min(kXferPiece, n - o), rec};
  };
  const uint64_t ha = (uint64_t)(uintptr_t)s.h_arena_dev, da = (uint64_t)(uintptr_t)s.d_arena;
  const uint64_t dr = (uint64_t)(uintptr_t)dres;
  for (const Pending &pd : s.reqs)
    if (pd.zc) add(pd.zc, da + pd.stage_off, pd.stage_len, ~0u);
    else if (kcopy) add(ha + pd.stage_off, da + pd.stage_off, pd.stage_len, ~0u);
  if (kcopy) add(ha + s.desc_off, da + s.desc_off, s.stat_off - s.desc_off, ~0u);
  // results: only for records whose status is 0 (complete_slot's rule)
  for (const Pending &pd : s.reqs)
    if (pd.zc)
      for (int q = 0; q < pd.nspan; ++q)
        add(dr + pd.stage_off + pd.span[q].stage_from, pd.zc + pd.span[q].stage_from, pd.span[q].n, pd.rec);
    else if (kcopy) add(dr + pd.stage_off, ha + pd.stage_off, pd.stage_len, pd.rec);
  if (kcopy) add(dr + s.stat_off, ha + s.stat_off, s.nrec, ~0u);
  const uint8_t *d_stat = dres + s.stat_off;

  if (!kcopy) {
    HIPCHK(c, hipMemcpyAsync(s.d_arena + in_lo, s.h_arena + in_lo, s.stat_off - in_lo, hipMemcpyHostToDevice, s_in));
    if (!small) {
      HIPCHK(c, hipEventRecord(s.in_done, s_in));
      HIPCHK(c, hipStreamWaitEvent(s_k, s.in_done, 0));
    }
  }
  if (nin && launch_xfer(s.h_xfer_dev, nin, nullptr, s_k)) return fail(c, ESPGPU_EIO, "xfer kernel launch failed");
  // kernel timing events (stats.kernel_ns, espgpu_last_kernel_ms) only on
  // large batches: on a burst's own stream each marker adds to its latency
  s.timed = !small || GPU_TIME_SMALL;
  if (s.timed) hipEventRecord(s.k0, s_k);
  // a single-session batch skips the device planner (ESPGPU_BATCH_GROUPED:
  // one session trivially satisfies "one session per chunk")
  int e = run_batch(c, s.d_arena, reinterpret_cast<const espgpu_desc *>(s.d_arena + s.desc_off), s.nrec,
                    dres + s.stat_off, s.op ? nullptr : s.d_out, s.mixed ? 0u : (uint32_t)ESPGPU_BATCH_GROUPED,
                    s.op, s_k, nullptr, s.kinds);
  if (e) return e;
  if (s.timed) hipEventRecord(s.k1, s_k);
  if (nout) s.wq = s_k;                          // results to host memory (zero-copy / staging)
  if (nout && launch_xfer(s.h_xfer_dev + nin, nout, d_stat, s_k)) return fail(c, ESPGPU_EIO, "xfer kernel launch failed");
  if (!kcopy) {
    if (!small) {
      HIPCHK(c, hipEventRecord(s.kout, s_k));
      HIPCHK(c, hipStreamWaitEvent(s_out, s.kout, 0));
    }
    HIPCHK(c, hipMemcpyAsync(s.h_arena + out_lo, dres + out_lo, out_hi - out_lo, hipMemcpyDeviceToHost, s_out));
  }
  HIPCHK(c, hipEventRecord(s.done, kcopy ? s_k : s_out));
  s.t_launch = now_ns();
  s.state = SLOT_INFLIGHT;
  c->stats.batches++;
  c->stats.zerocopy += s.nrec - s.nstaged;
  c->cur = (c->cur + 1) % (int)c->slots.size();
  return 0;
}

int espgpu_flush(espgpu_ctx *c) {
  if (!c) return ESPGPU_EINVAL;
  if (c->failed) return ESPGPU_EIO;
  // the filling slot, then the overflow (oldest first) into the free slots
  Overflow &o = c->ovf;
  for (;;) {
    Slot &s = c->slots[c->cur];
    if (s.state == SLOT_FILLING) {
      // a batch that cannot be launched is a GPU failure: its requests, the
      // overflow's and (through poll) the in-flight ones complete with EIO
      if (launch_slot(c, s)) return fail_launch(c, s);
      continue;
    }
    if (o.empty() || s.state != SLOT_FREE) break;
    while (!o.empty()) {
      const OvfEntry &en = o.front();
      if (slot_full(c, s, en.op, en.pd.stage_len)) break;
      if (!en.pd.zc) memcpy(s.h_arena + s.bytes, o.bytes.buf.get() + en.pd.stage_off, en.pd.stage_len);
      slot_commit(s, en.pd, en.d, o.segpool.buf.get() + en.pd.seg0, en.sid, en.op, en.kind);
      o.pop();
    }
  }
  return 0;
}

static int complete_slot(espgpu_ctx *c, Slot &s) {
  float ms = 0.f;
  if (s.timed && hipEventElapsedTime(&ms, s.k0, s.k1) == hipSuccess) {
    c->last_ms = ms;
    c->stats.kernel_ns += (uint64_t)(ms * 1e6);
  }
  for (auto &pd : s.reqs) {
    int et = pd.etype_pre >= 0 ? pd.etype_pre : (int)s.h_arena[s.stat_off + pd.rec];
    if (et == 0) {
      const uint8_t *src = s.h_arena + pd.stage_off;
      for (int k = 0; k < pd.nspan && !pd.zc; ++k)     // zero-copy: the xfer kernel wrote them
        seg_copy_in(s.segpool.data() + pd.seg0, pd.nsegs, pd.span[k].buf_off, pd.span[k].n,
                    src + pd.span[k].stage_from);
      c->stats.bytes += pd.span[0].n;
    } else if (et == ESPGPU_EBADMSG) {
      c->stats.auth_fail++;
    } else {
      c->stats.einval++;
    }
    c->stats.records++;
    c->ready.push_back(espgpu_completion{pd.opaque, et});
  }
  s.reqs.clear();
  s.segpool.clear();
  s.nrec = 0;
  s.bytes = 0;
  s.state = SLOT_FREE;
  return 0;
}

int espgpu_poll(espgpu_ctx *c, espgpu_completion *out, int max) {
  if (!c) return -ESPGPU_EINVAL;
  // completions of flushed batches, oldest first, and in arrival order: a
  // batch that finished before an older one (another stream's kernel, a
  // doorbell job another workgroup took) waits for it
  // (a batch whose completion fails, or that outlives deadline_ms, fails the
  // ctx and completes with EIO: slot_check)
  bool door_wait = false;
  const uint64_t now = now_ns();
  for (size_t k = 0; k < c->slots.size(); ++k) {
    Slot &s = c->slots[(c->cur + k) % c->slots.size()];
    if (s.state != SLOT_INFLIGHT) continue;
    const int r = slot_check(c, s, now);
    if (r == 0) {
      // a doorbell job outstanding for over 100 us: make sure the kernel is
      // still there (a workgroup that read a retire request just before the
      // job was published may have exited with it)
      door_wait = s.door_job >= 0 && now - s.door_t0 > 100000u;
      break;
    }
    if (r < 0) {
      drop_slot(c, s);
      continue;
    }
    s.door_job = -1;
    complete_slot(c, s);
  }
  if (door_wait && !c->failed && door_ensure(c)) ctx_fail(c, "door kernel relaunch failed");
  const int avail = (int)(c->ready.size() - c->ready_head);
  const int n = std::min(max, avail);
  for (int i = 0; i < n; ++i) out[i] = c->ready[c->ready_head + i];
  c->ready_head += n;
  if (c->ready_head == c->ready.size()) {
    c->ready.clear();
    c->ready_head = 0;
  }
  return n;
}

int espgpu_drain(espgpu_ctx *c) {
  if (!c) return ESPGPU_EINVAL;
  do {
    espgpu_flush(c);              // (a launch failure fails the ctx: the loop below retires the rest)
    // oldest first (slot cur is the next to fill, so cur+1.. are older
    // batches); every wait is bounded by deadline_ms (slot_check), so a
    // batch the GPU never finishes completes with EIO instead of hanging
    for (size_t k = 0; k < c->slots.size(); ++k) {
      Slot &s = c->slots[(c->cur + k) % c->slots.size()];
      if (s.state != SLOT_INFLIGHT) continue;
      int r;
      while ((r = slot_check(c, s, now_ns())) == 0) {
        // the persistent kernel's job: relaunch the kernel if it exited
        if (s.door_job >= 0 && !c->failed && door_ensure(c)) ctx_fail(c, "door kernel relaunch failed");
        sched_yield();
      }
      if (r < 0) {
        drop_slot(c, s);
        continue;
      }
      s.door_job = -1;
      complete_slot(c, s);
    }
  } while (!c->ovf.empty());     // the overflow goes into the slots just freed
  return c->failed ? ESPGPU_EIO : 0;
}

int espgpu_register_host(espgpu_ctx *c, void *base, uint64_t len) {
  if (!c || !base || !len) return ESPGPU_EINVAL;
  const uintptr_t b = (uintptr_t)base;
  for (const HostRegion &r : c->regions)
    if (b < r.base + r.len && r.base < b + len) return fail(c, ESPGPU_EINVAL, "overlaps a registered region");
  bool owned = true;
  hipError_t e = hipHostRegister(base, len, hipHostRegisterMapped);
  if (e == hipErrorHostMemoryAlreadyRegistered) {
    owned = false;                   // already pinned (hipHostMalloc): only map it
    (void)hipGetLastError();
  } else if (e != hipSuccess) {
    return fail(c, ESPGPU_EIO, "hipHostRegister: %s", hipGetErrorString(e));
  }
  void *dp = nullptr;
  if (hipHostGetDevicePointer(&dp, base, 0) != hipSuccess || !dp) {
    if (owned) hipHostUnregister(base);
    return fail(c, ESPGPU_EIO, "hipHostGetDevicePointer failed");
  }
  HostRegion r{b, len, (uint64_t)(uintptr_t)dp, owned};
  c->regions.insert(std::upper_bound(c->regions.begin(), c->regions.end(), r,
                                     [](const HostRegion &x, const HostRegion &y) { return x.base < y.base; }),
                    r);
  return 0;
}

int espgpu_unregister_host(espgpu_ctx *c, void *base) {
  if (!c) return ESPGPU_EINVAL;
  auto it = std::find_if(c->regions.begin(), c->regions.end(),
                         [&](const HostRegion &r) { return r.base == (uintptr_t)base; });
  if (it == c->regions.end()) return ESPGPU_EINVAL;
  // requests staged from it run to completion first (their completions wait for poll)
  int e = espgpu_drain(c);
  if (e) return e;
  if (it->owned) hipHostUnregister(base);
  c->regions.erase(it);
  return 0;
}

int espgpu_replay_params_ok(const espgpu_replay *r) {
  if (!r) return 0;
  if (r->wsize == 0) return 1;
  const uint32_t b = r->bitmap_size;
  return b != 0 && (b & (b - 1)) == 0 && (uint64_t)b * 32 >= (uint64_t)r->wsize * 8;
}

int espgpu_replay_check_batch(espgpu_ctx *c, const uint8_t *d_arena, espgpu_desc *d_desc, uint32_t n,
                              const espgpu_replay *d_replay, uint32_t nreplay, const uint32_t *d_bitmap,
                              uint8_t *d_rstatus, void *stream) {
  if (!c || (n && (!d_arena || !d_desc || !d_rstatus || (nreplay && (!d_replay || !d_bitmap)))))
    return ESPGPU_EINVAL;
  if (launch_replay_check(d_arena, d_desc, n, d_replay, nreplay, d_bitmap, d_rstatus, stream))
    return fail(c, ESPGPU_EIO, "replay check kernel launch failed");
  return 0;
}

int espgpu_replay_merge(espgpu_ctx *c, uint8_t *d_status, const uint8_t *d_rstatus, uint32_t n, void *stream) {
  if (!c || (n && (!d_status || !d_rstatus))) return ESPGPU_EINVAL;
  if (launch_replay_merge(d_status, d_rstatus, n, stream))
    return fail(c, ESPGPU_EIO, "replay merge kernel launch failed");
  return 0;
}

// ipsec_updatereplay (freebsd/netipsec/ipsec.c:1338-1436) with the window
// helpers advance_window / set_window (:1203-1232): after authentication, in
// arrival order per SA.
int espgpu_replay_update(espgpu_replay *r, uint32_t *bitmap, uint32_t seq) {
  if (!r || (r->wsize && !bitmap)) return ESPGPU_EINVAL;
  if (r->wsize == 0) return 0;
  // the window indexes the bitmap with bitmap_size - 1 as a mask: a power of
  // two covering wsize * 8 bits (key.c:3346-3351 sizes it so)
  if (!espgpu_replay_params_ok(r)) return ESPGPU_EINVAL;
  if (seq == 0 && r->last == 0) return ESPGPU_EACCES;
  uint32_t *bm = bitmap + r->bitmap_off;
  const uint32_t mask = r->bitmap_size - 1;
  auto seen = [&](uint32_t s) { return (bm[(s >> 5) & mask] >> (s & 31)) & 1u; };
  auto mark = [&](uint32_t s) { bm[(s >> 5) & mask] |= 1u << (s & 31); };
  auto advance = [&](uint64_t s) {      // clear the words the window top moves past
    const uint64_t cur = r->last >> 5;
    uint64_t diff = (s >> 5) - cur;
    if (diff > r->bitmap_size) diff = r->bitmap_size;
    for (uint64_t k = 0; k < diff; ++k) bm[(k + cur + 1) & mask] = 0;
  };
  const uint32_t window = r->wsize << 3;
  const uint32_t tl = (uint32_t)r->last, th = (uint32_t)(r->last >> 32);
  const uint32_t bl = tl - window + 1;
  if ((tl >= window - 1 && seq >= bl) || (tl < window - 1 && seq < bl)) {
    if (seq <= tl) {
      if (seen(seq)) return ESPGPU_EACCES;
      mark(seq);
    } else {
      const uint64_t s = ((uint64_t)th << 32) | seq;
      advance(s);
      mark(seq);
      r->last = s;
    }
    return 0;
  }
  if (!(r->flags & ESPGPU_REPLAY_ESN)) return ESPGPU_EACCES;
  if (tl < window - 1 && seq >= bl) {   // in the window, previous subspace
    if (th == 0 || seen(seq)) return ESPGPU_EACCES;
    mark(seq);
    return 0;
  }
  if (th + 1 == 0) return ESPGPU_EACCES;   // the high part would wrap
  const uint64_t s = ((uint64_t)(th + 1) << 32) | seq;
  advance(s);
  mark(seq);
  r->last = s;
  return 0;
}

int espgpu_get_stats(espgpu_ctx *c, espgpu_stats *st) {
  if (!c || !st) return ESPGPU_EINVAL;
  *st = c->stats;
  st->ovf_reserved = c->ovf.reserved();
  st->ovf_peak = c->ovf.peak_bytes;
  return 0;
}

// The device-resident entry points: a launch that could not be queued (EIO)
// fails the ctx as a process-path launch does (later calls answer EIO).
static int batch_rc(espgpu_ctx *c, int e) {
  if (e == ESPGPU_EIO && !c->failed) ctx_fail(c, "batch launch failed");
  return e;
}

int espgpu_decrypt_batch(espgpu_ctx *c, uint8_t *d_arena, const espgpu_desc *d_desc, uint32_t n,
                         uint8_t *d_status, uint8_t *d_out, uint32_t flags, void *stream) {
  if (!c || (!d_arena && n) || (!d_desc && n) || (!d_status && n)) return ESPGPU_EINVAL;
  return batch_rc(c, run_batch(c, d_arena, d_desc, n, d_status, d_out ? d_out : d_arena, flags, 0,
                             reinterpret_cast<hipStream_t>(stream)));
}

int espgpu_decrypt_batch_trailer(espgpu_ctx *c, uint8_t *d_arena, const espgpu_desc *d_desc,
                                 uint32_t n, uint8_t *d_status, uint8_t *d_out, uint32_t *d_trailer,
                                 uint32_t flags, void *stream) {
  if (!c || (!d_arena && n) || (!d_desc && n) || (!d_status && n) || (!d_trailer && n)) return ESPGPU_EINVAL;
  return batch_rc(c, run_batch(c, d_arena, d_desc, n, d_status, d_out ? d_out : d_arena, flags, 0,
                             reinterpret_cast<hipStream_t>(stream), d_trailer));
}

int espgpu_decrypt_batch_packed(espgpu_ctx *c, uint8_t *d_arena, const espgpu_desc *d_desc, uint32_t n,
                                uint8_t *d_status, uint8_t *d_out, uint32_t out_stride, uint32_t flags,
                                void *stream) {
  if (!c || (!d_arena && n) || (!d_desc && n) || (!d_status && n) || (!d_out && n) || d_out == d_arena ||
      out_stride == 0 || out_stride % 128 != 0 || ((uintptr_t)d_out & 127))
    return ESPGPU_EINVAL;
  return batch_rc(c, run_batch(c, d_arena, d_desc, n, d_status, d_out, flags, 0, reinterpret_cast<hipStream_t>(stream),
                             nullptr, 3, nullptr, out_stride));
}

int espgpu_encrypt_batch(espgpu_ctx *c, uint8_t *d_arena, const espgpu_desc *d_desc, uint32_t n,
                         uint8_t *d_status, uint32_t flags, void *stream) {
  if (!c || (!d_arena && n) || (!d_desc && n) || (!d_status && n)) return ESPGPU_EINVAL;
  return batch_rc(c, run_batch(c, d_arena, d_desc, n, d_status, nullptr, flags, 1, reinterpret_cast<hipStream_t>(stream)));
}

float espgpu_last_kernel_ms(espgpu_ctx *c) { return c ? c->last_ms : 0.f; }

static int host_pipeline(espgpu_ctx *c, const uint8_t *h_arena, uint64_t arena_bytes,
                         const espgpu_desc *h_desc, uint32_t n, uint8_t *h_status, uint8_t *h_out,
                         uint32_t chunk, uint32_t flags, int encrypt) {
  if (!c || !h_arena || !h_desc || !h_status || (!encrypt && !h_out)) return ESPGPU_EINVAL;
  if (n == 0) return 0;
  if (!chunk) chunk = 65536;
  if (arena_bytes + 64 > c->e2e_bytes || n > c->e2e_n) {
    hipFree(c->e2e_arena); hipFree(c->e2e_out); hipFree(c->e2e_status); hipFree(c->e2e_desc);
    c->e2e_bytes = arena_bytes + 64;
    c->e2e_n = n;
    HIPCHK(c, hipMalloc(&c->e2e_arena, c->e2e_bytes));
    HIPCHK(c, hipMalloc(&c->e2e_out, c->e2e_bytes));
    HIPCHK(c, hipMalloc(&c->e2e_status, n));
    HIPCHK(c, hipMalloc(&c->e2e_desc, (size_t)n * sizeof(espgpu_desc)));
  }
  // Chunks of consecutive records (descriptors in ascending arena order) map to
  // contiguous byte ranges, copied to the same offsets of a device mirror so the
  // descriptors are used unchanged.
  for (uint32_t i0 = 0, k = 0; i0 < n; i0 += chunk, ++k) {
    const uint32_t i1 = std::min(n, i0 + chunk), m = i1 - i0;
    uint64_t lo = (uint64_t)h_desc[i0].off4 * 4, hi = 0;
    for (uint32_t i = i0; i < i1; ++i) {
      const uint64_t o = (uint64_t)h_desc[i].off4 * 4;
      lo = std::min(lo, o);
      hi = std::max(hi, o + h_desc[i].len);
    }
    hi = std::min(arena_bytes, hi + 16);                 // partial-block loads read <= 16 B past
    hipEvent_t ein = c->e2e_in[k & 1], ek = c->e2e_k[k & 1];
    HIPCHK(c, hipMemcpyAsync(c->e2e_desc + i0, h_desc + i0, m * sizeof(espgpu_desc), hipMemcpyHostToDevice, c->s_in));
    HIPCHK(c, hipMemcpyAsync(c->e2e_arena + lo, h_arena + lo, hi - lo, hipMemcpyHostToDevice, c->s_in));
    HIPCHK(c, hipEventRecord(ein, c->s_in));
    HIPCHK(c, hipStreamWaitEvent(c->stream, ein, 0));
    int e = run_batch(c, c->e2e_arena, c->e2e_desc + i0, m, c->e2e_status + i0,
                      encrypt ? nullptr : c->e2e_out, flags, encrypt, c->stream);
    if (e) return e;
    HIPCHK(c, hipEventRecord(ek, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->s_out, ek, 0));
    uint8_t *dst = encrypt ? (uint8_t *)h_arena : h_out;
    HIPCHK(c, hipMemcpyAsync(dst + lo, (encrypt ? c->e2e_arena : c->e2e_out) + lo, hi - lo, hipMemcpyDeviceToHost, c->s_out));
    HIPCHK(c, hipMemcpyAsync(h_status + i0, c->e2e_status + i0, m, hipMemcpyDeviceToHost, c->s_out));
  }
  HIPCHK(c, hipStreamSynchronize(c->s_out));
  return 0;
}

int espgpu_decrypt_host(espgpu_ctx *c, const uint8_t *h_arena, uint64_t arena_bytes,
                        const espgpu_desc *h_desc, uint32_t n, uint8_t *h_status, uint8_t *h_out,
                        uint32_t chunk, uint32_t flags) {
  if (c && c->failed) return ESPGPU_EIO;
  return batch_rc(c, host_pipeline(c, h_arena, arena_bytes, h_desc, n, h_status, h_out, chunk, flags, 0));
}

int espgpu_set_tuning(espgpu_ctx *c, const char *key, int value) {
  if (!c || !key) return ESPGPU_EINVAL;
  if (!strcmp(key, "grid")) { c->cfg.grid = (uint32_t)value; return 0; }
  if (!strcmp(key, "gcm_lanes")) {
    if (value != 0 && value != kGcmLanesPerRec && value != kGcmLanesSmall) return ESPGPU_EINVAL;
    c->gcm_lanes = value;
    return 0;
  }
  if (!strcmp(key, "overflow_mb")) {
    // offsets into the overflow's byte buffer are 32-bit (Pending::stage_off)
    if (value < 0 || value > 4095) return ESPGPU_EINVAL;
    // the rings are reserved whole here: growing the overflow inside
    // process() would copy it (hundreds of microseconds at a few MiB).
    // Resizing drains what the old rings hold first.
    if (!c->ovf.empty()) {
      int e = espgpu_drain(c);
      if (e) return e;
    }
    // all three rings or none: on ENOMEM the previous overflow stays
    if (!c->ovf.init((size_t)value << 20))
      return fail(c, ESPGPU_ENOMEM, "overflow_mb %d: host allocation failed", value);
    c->ovf_cap = (size_t)value << 20;
    return 0;
  }
  if (!strcmp(key, "fault")) {
    // fault injection (tests of the GPU-failure path): ESPGPU_FAULT_* bits,
    // each consumed by the next launch / completion query / launched batch
    if (value & ~(ESPGPU_FAULT_LAUNCH | ESPGPU_FAULT_QUERY | ESPGPU_FAULT_STUCK)) return ESPGPU_EINVAL;
    c->fault = (uint32_t)value;
    return 0;
  }
  if (!strcmp(key, "deadline_ms")) {
    if (value < 1 || value > 600000) return ESPGPU_EINVAL;
    c->deadline_ms = (uint32_t)value;
    return 0;
  }
  if (!strcmp(key, "gcm_burst")) {
    if (value < 0) return ESPGPU_EINVAL;
    c->gcm_burst = (uint32_t)value;
    return 0;
  }
  if (!strcmp(key, "stage_fused")) {
    if (value != 0 && value != 1) return ESPGPU_EINVAL;
    c->stage_fused = value;
    return 0;
  }
  if (!strcmp(key, "xfer")) {
    if (value != 0 && value != 1) return ESPGPU_EINVAL;
    c->xfer_small = value;
    return 0;
  }
  if (!strcmp(key, "door")) {
    // workgroups of the doorbell kernel (0 = off); changing it drains and
    // stops the running kernel (the next batch relaunches it)
    if (value < 0 || value > 256) return ESPGPU_EINVAL;
    if (value != c->door_wg && c->door_ctl) {
      int e = espgpu_drain(c);
      if (e) return e;
      door_stop(c);
    }
    c->door_wg = value;
    return value ? door_setup(c) : 0;
  }
  if (!strcmp(key, "door_idle_us")) {
    if (value < 100 || value > 10000000) return ESPGPU_EINVAL;
    door_stop(c);
    c->door_idle_us = (uint32_t)value;
    return 0;
  }
  if (!strcmp(key, "gcm_opts")) return set_gcm_opts((uint32_t)value) ? ESPGPU_ENOTSUP : 0;
  if (!strcmp(key, "eta_opts")) return set_eta_opts((uint32_t)value) ? ESPGPU_ENOTSUP : 0;
  return ESPGPU_ENOENT;
}

}  // extern "C"
