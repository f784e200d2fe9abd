// espgpu_internal.h — device-side data layouts shared by the host runtime
// (espgpu.cpp) and the HIP kernels (esp_gcm.hip, esp_cbc.hip, plan.hip,
// xfer.hip).
#pragma once
#include <stdint.h>

#include "espgpu.h"

namespace espgpu {

// ---- per-SA device record (one per session slot), 1 KiB ----------------------
// GCM: rk[] is the AES encryption schedule in "kernel form" for the pair-table
//   round (esp_gcm.hip): rk[0..3] raw, rk[4r..4r+3] = ror16(rk) for the
//   middle rounds, rk[4nr..] byte-swapped (the last round emits little-endian
//   words); dk[] unused.  The GHASH tables live in a separate array.
// ETA: rk[] = encryption schedule (raw, big-endian words, rijndael-alg-fst.c
//   layout), dk[] = decryption schedule (rijndaelKeySetupDec layout), ipad/opad
//   = SHA-1 chaining state after one block of key^0x36 / key^0x5c
//   (hmac_init_pad, crypto.c:413-441).  CSP_MODE_CIPHER sessions are ETA
//   sessions to the kernels (mode ETA) with aalg 0 and mlen 0: the cipher pass
//   alone; calg ESPGPU_CRYPTO_NULL_CBC is the identity cipher (no key, no IV).
struct DevSA {
  uint32_t rk[64];
  uint32_t dk[64];
  uint32_t nr;
  uint32_t mode;    // ESPGPU_CSP_MODE_AEAD / _ETA, 0 = free slot
  uint32_t flags;   // csp_flags
  uint32_t mlen;    // ICV bytes compared / written
  uint32_t ipad[16]; // ETA: HMAC chaining states after the ipad / opad key
  uint32_t opad[16]; //      block (5 words SHA-1, 8 SHA2-256, 16 SHA2-384/512:
                     //      64-bit state word k as words 2k (high), 2k+1)
  uint32_t calg;    // ETA cipher: ESPGPU_CRYPTO_AES_CBC, _AES_ICM (CTR) or _NULL_CBC
  uint32_t aalg;    // ETA auth: ESPGPU_CRYPTO_SHA1_HMAC or _SHA2_256/384/512_HMAC, 0 = none
  uint32_t pad_[256 - 128 - 4 - 32 - 2];
};
static_assert(sizeof(DevSA) == 1024, "DevSA is 1 KiB");

// GHASH multiplication tables for one SA (host_crypto.cpp ghash_tables):
// H^1..H^8 with 4-bit indices, 8 KiB per power (power e at (e-1)*8 KiB):
// nibble position j (byte j>>1 of the block in memory order, low nibble if j
// even), value n at j*256 + n*16.  Read from L2 by the per-record final
// multiply by H^(S-l), and expanded by a workgroup into the 8-bit table of
// its Horner multiplier H^S in LDS (esp_gcm.hip stage_h8: byte position p,
// value v at v*256 + p*16, value-major so a row's 16 positions sit in the 16
// bank quads; gf_mul8) whenever it changes session.
constexpr int kGcmLanesPerRec = 4;                               // GCM kernel: lanes per record
constexpr int kGcmLanesSmall = 8;                                // small batches: shorter serial chain
constexpr uint32_t kGcmSmallBatch = 32768;                       // records: below, 8 lanes per record still fit the chip
constexpr uint32_t kGhPowerBytes = 32 * 16 * 16;                 // 8192
constexpr uint32_t kGh8Bytes = 16 * 256 * 16;                    // 65536: an 8-bit table (LDS only)
constexpr uint32_t kGhTableBytes = 8 * kGhPowerBytes;            // 65536 per SA

// A chunk: up to kChunkRecs records of ONE session, processed by one
// workgroup iteration of the GCM kernel.  rec positions index `order`
// (or the descriptor array directly when order == nullptr).
constexpr int kChunkRecs = 256;
struct Chunk {
  uint32_t sa;
  uint32_t start;
  uint32_t count;
  uint32_t cls;     // size class 0..3 (GCM), 4 = invalid-session or ETA chunk
};

struct GcmParams {
  uint8_t *arena;                 // records (read; written in place for encrypt)
  uint8_t *out;                   // decrypt output (may == arena)
  const espgpu_desc *desc;
  const uint32_t *order;          // planner permutation or nullptr
  const Chunk *chunks;            // explicit chunk list, or nullptr (implicit)
  const uint32_t *nchunks;        // [0] = GCM (+invalid) chunks, [1] = all chunks
  uint32_t n;                     // number of descriptors (implicit mode)
  const DevSA *sas;
  const uint8_t *gtab;            // [slot][kGhTableBytes]
  const uint2 *tpair;             // 256 x (Te0[x], Te1[x])
  uint8_t *status;
  uint32_t nsas;
  // Work queue: [0] next chunk ticket, [1] retired workgroups.  Zero before a
  // launch; the last workgroup to retire resets both, so no per-launch memset.
  // Launches sharing a ctx must be stream-ordered (as the planner workspace).
  uint32_t *queue;
  uint32_t *trailer;              // decrypt: fused esp_input_cb trailer words, or nullptr
  uint32_t chunk;                 // implicit mode: records per chunk (launch_gcm sets it)
  uint4 *ej0;                     // burst design: E_K(J0) per descriptor (nullptr: fused kernel)
  // A small single-session process batch that stages its own records (one
  // kernel instead of copy, kernel, copy): per descriptor i, xin[i] copies the
  // record into the arena before its chunk runs and xout[2i], xout[2i+1] copy
  // its results back after (len 0: none; only if its status is 0); hstat is
  // the host status array; hdesc the host descriptors, which each chunk
  // copies to desc (device) with its records.  nullptr: the records are in
  // the arena already.
  const struct XferSpan *xin, *xout;
  uint8_t *hstat;
  const espgpu_desc *hdesc;
  // decrypt out of place: 0 = plaintext at the record's own offset in out;
  // else record i's plaintext at out + i * out_stride (espgpu_decrypt_batch_packed)
  uint32_t out_stride;
};

// Work-queue regions (ctx d_queue): one per kernel family, kQueueRegionWords
// apart.  Word 0 = the ticket counter, word 1 = retired count.
constexpr uint32_t kQueueRegionWords = 1024;

struct EtaParams {
  uint8_t *arena;
  uint8_t *out;
  const espgpu_desc *desc;
  const uint32_t *order;          // planner permutation or nullptr (implicit)
  const Chunk *chunks;            // ETA chunks are [nchunks[0], nchunks[1])
  const uint32_t *nchunks;
  uint32_t *queue;                // [0] ticket, [1] retired waves (self-resetting)
  uint32_t *trailer;              // decrypt: fused esp_input_cb trailer words, or nullptr
  uint32_t n;
  const DevSA *sas;
  const uint2 *tpair;             // encryption pair table
  const uint2 *dpair;             // decryption pair table (Td0, Td1)
  const uint8_t *isbox;           // inverse S-box (256 B)
  uint8_t *status;
  uint32_t nsas;
};

// esp_input_cb's checks on the last 3 plaintext bytes (xform_esp.c:597-630),
// given the 4-byte-aligned dword holding them (bytes 1..3 in memory order)
// and the payload (ESP ciphertext) length.  Bits as ESPGPU_TR_* (espgpu.h).
__host__ __device__ inline uint32_t esp_trailer_word(uint32_t wlast, uint32_t plen) {
  const uint32_t l0 = (wlast >> 8) & 0xffu, padlen = (wlast >> 16) & 0xffu, nh = wlast >> 24;
  uint32_t t = nh | (padlen << 8) | ESPGPU_TR_VALID;
  if (padlen + 2 > plen) t |= ESPGPU_TR_BADLEN;
  if (padlen != l0 && padlen != 0) t |= ESPGPU_TR_BADPAD;
  if (nh == 59) t |= ESPGPU_TR_NONE;                       // IPPROTO_NONE
  return t;
}

// One copy of the opencrypto path's staging transfers (xfer.hip): len bytes
// from src to dst (device or host-mapped addresses); rec != ~0u: only if
// status[rec] == 0.  The host splits spans into pieces of at most kXferPiece
// bytes, one workgroup each.
struct XferSpan {
  uint64_t src, dst;
  uint32_t len, rec;
};
constexpr uint32_t kXferPiece = 4096;

// ---- doorbell burst path (set_tuning "door", esp_gcm.hip gcm_door_kernel) ----
// A persistent kernel of `door` workgroups (one per CU) serves the process
// path's single-session GCM bursts without a launch per burst: flush writes a
// 16-byte job into a ring in pinned host memory, the workgroups poll it over
// the mapping, claim the job's chunks from a device counter, stage the
// records in and the results out as the burst kernel does, and the workgroup
// finishing a job's last chunk writes its number into done[] (host memory),
// which poll() reads.  The kernel exits when the host sets stop or after
// idle_ticks of s_memrealtime (100 MHz) without a job; poll() relaunches it
// when a job is outstanding and it has exited.
constexpr uint32_t kDoorRing = 64;              // job ring entries (>= staging slots)
struct DoorJob {                                 // host-written; seq last (= job number + 1)
  uint32_t n;                                    // records
  uint32_t slot_op;                              // staging slot | op << 16 (0 decrypt, 1 encrypt)
  uint32_t chk;                                  // n ^ slot_op ^ seq ^ kDoorChk: a torn read never matches
  uint32_t seq;
};
constexpr uint32_t kDoorChk = 0x5eed1e55u;
constexpr uint32_t kDoorStopNow = 1;             // DoorCtl::stop: exit between chunks
constexpr uint32_t kDoorStopIdle = 2;            // exit once no published job is waiting
struct DoorCtl {                                 // pinned host memory, device-mapped
  DoorJob ring[kDoorRing];
  uint32_t stop;                                 // 0, kDoorStopNow or kDoorStopIdle
  uint32_t pad_[31];
  uint32_t done[kDoorRing];                      // job number + 1 once the job completed
};
struct DoorDev {                                 // device memory, zeroed once
  // per ring entry: (job + 1) << 32 | chunks claimed.  A workgroup installs
  // job j's generation (CAS from an older one) only after it has seen job j
  // published, then claims with an atomic add; an add that lands on a later
  // job's generation holds that job's chunk (it is published), so no claim
  // is ever lost and none waits on an unpublished job.
  unsigned long long tick[kDoorRing];
  uint32_t fin[kDoorRing];                       // chunks finished, per ring entry
  uint32_t next;                                 // lowest job not known to be fully claimed (a hint)
};
struct DoorSlot {                                // per staging slot (device table)
  uint8_t *arena, *out;                          // out: decrypt results (encrypt: in place)
  uint4 *ej0;
  const struct XferSpan *xin, *xout;             // xin[i]; xout[2i], xout[2i+1]
  uint8_t *hdesc, *hstat;                        // host descriptors / statuses (mapped)
  uint32_t desc_off, stat_off;                   // device descriptors and statuses in arena / out
};
struct DoorArgs {
  DoorCtl *ctl;                                  // device-mapped address
  DoorDev *dev;
  const DoorSlot *slots;
  uint32_t nslots;
  uint32_t chunk;                                // records per chunk
  uint32_t idle_ticks;
  const DevSA *sas;
  const uint8_t *gtab;
  const uint2 *tpair;
  uint32_t nsas;
};

// Launchers (defined in the .hip files, called by espgpu.cpp).
int launch_gcm_door(const DoorArgs &a, int grid, void *stream);
// lanes: 0 = by batch size (kGcmLanesSmall below kGcmSmallBatch records,
// else kGcmLanesPerRec), or force 4 / 8 (set_tuning "gcm_lanes", tests)
int launch_gcm(const GcmParams &p, int encrypt, int two_pass, int grid, int lanes, void *stream);
int set_gcm_opts(uint32_t opts);   // measurement knobs (`make knobs` builds only)
int set_eta_opts(uint32_t opts);
// kinds: bit 0 = SHA-1 / SHA2-256 / no-auth CBC sessions in the SA table,
// bit 1 = such CTR (or ESP-NULL) ones, bits 2 / 3 = SHA2-384/512 CBC / CTR
// ones, bit 4 = any SHA2-384/512 session
int launch_eta(const EtaParams &p, int encrypt, int kinds, int grid, void *stream);
int launch_replay_check(const uint8_t *arena, espgpu_desc *desc, uint32_t n, const espgpu_replay *rp,
                        uint32_t nrp, const uint32_t *bitmap, uint8_t *rstatus, void *stream);
int launch_xfer(const XferSpan *spans, uint32_t nspans, const uint8_t *status, void *stream);
int launch_replay_merge(uint8_t *status, const uint8_t *rstatus, uint32_t n, void *stream);
int launch_plan(const espgpu_desc *d_desc, uint32_t n, const DevSA *sas, uint32_t nsas, uint32_t cap_sas,
                uint32_t *d_work, uint32_t *d_order, Chunk *d_chunks, uint32_t *d_nchunks,
                uint32_t max_chunks, void *stream);
size_t plan_workspace_words(uint32_t nsas);
uint32_t plan_max_chunks(uint32_t n, uint32_t nsas);

}  // namespace espgpu
