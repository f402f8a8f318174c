// xyws_stream.hip — run-parallel stream decoder for gfx950 (the default mode
// of xyws_decode_stream).
//
// The problem: in a back-to-back batch the start of frame k+1 is known only
// once the header of frame k is parsed (websocket_frame_header.h:305-385 gives
// header size and payload length), so frame boundaries form a linked list
// through the batch, and websocket_mask (websocket_frame_mask.h:6-25) can only
// run on a payload once its frame is found.
//
// Geometry (measured, scripts/bw_probe.hip): the in-place XOR of a 2 GiB batch
// runs at 5.98 TB/s (R+W) with one 1024-thread workgroup per CU, each streaming
// its own contiguous byte range in 128 KiB SEGMENTS staged in LDS, nontemporal
// 16-byte buffer loads/stores and a one-segment register prefetch. This kernel
// is that data movement plus the header chase:
//
//  * The batch is cut into RUNS of equal byte ranges, one per workgroup (a ticket
//    gives runs out in dispatch order).
//  * Inside a run the chase is EXACT and serial: lane 0 parses each header from
//    the LDS copy of the segment and appends (payload range, rotated key word) to
//    a frame list; then every lane XORs its 16-byte chunks with the listed keys
//    and stores them. No speculation, no waiting, inside a run.
//  * A run r > 0 does not know where the chain enters it. Its prologue takes the
//    earliest position whose chain of KHDR headers is plausible for a client
//    stream (RSV = 0, known opcode, control frames short with FIN, MASK as
//    expected, minimal length encoding) and publishes it as h_r (for a 7-bit
//    length form, the next node instead: a false short "header" just before a
//    true one lands exactly on it, the next node is then true either way), with
//    its write start W_r = round16(h_r + header). Run r writes bytes >= W_r,
//    run r-1 writes bytes < W_r: run r-1 keeps chasing past its range until its
//    exact chain reaches h_r and XORs the bytes up to W_r. If its chain lands
//    exactly on h_r, run r's entry is exact; by induction from run 0 (exact:
//    batch start and carry) every run is exact when every boundary matches.
//  * A mismatch (rare: an implausible true header, or a plausible false chain)
//    is repaired by finish_call: undo the mis-speculated run (replaying its
//    own chain XORs its payloads back; a chain never writes its own headers),
//    then redo its range from the exact chain, boundary after boundary until the
//    chains agree again. Speculation decides speed only: any byte stream (RSV
//    bits, reserved opcodes, unmasked or non-minimal frames, random bytes)
//    decodes exactly as the reference parses it.
//
// The only inter-workgroup hand-off is a run's published (h, W): sc1 record
// stores, s_waitcnt vmcnt(0), one agent-scope flag store; the reader polls the
// flag with sc1 loads and reads the record with sc1 loads
// (MI355X_MICROARCH.md §Workgroup dispatch, valid forms). A run waits only for
// the prologue of the next run with an entry, whose ticket was taken after its
// own and which never waits, so the lowest ticket always progresses. Header
// bytes are read only where no other workgroup writes: below the successor's W
// (a header that would cross it stops the chase, "cut"), or in the run's own
// range. Flags and the ticket are zeroed when scratch is allocated and reset by
// finish_call after every call (so a captured graph replays correctly);
// spins are bounded and report through the device error word.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>
#include <mutex>
#include <cstdlib>

#include "xyws_stream.h"
#include "xyws_device.h"
#include "xyws_ctx.h"  // (zero_now)

namespace {



constexpr uint64_t NONE = ~0ull;
constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr uint32_t PAD = 32;          // LDS bytes after the segment (5-dword header reads)
// Headers a speculative entry's chain must pass, by the entry's length form:
// a false 127-form header needs 0xFF/0x7F plus an 8-byte length below 2^46
// (~3e-10 per random position), a 126-form one 0xFE/0x7E (~9e-5), a 7-bit
// one a plausible first byte and mask bit (~2.3e-2); each further plausible
// header multiplies by ~2.3e-2. A prologue scans up to a few MB of payload
// when frames are large (2^28 positions per call over all runs at 1 MiB
// frames), so a false chain costs ~1e-12 per position (127 form: ~8e-12, two
// headers, the second one mostly still in LDS for 64 KiB frames): ~1e-3 per
// call at worst. Short hops stay in LDS; long ones are memory reads (batched
// after the scan). A false entry costs time (a repair), never bytes.
constexpr uint32_t KHDR_127 = 2, KHDR_126 = 6, KHDR_7 = 8;
constexpr uint32_t SPIN = 1u << 24;   // bounded spins (s_sleep 2 each: ~1 s)
constexpr uint32_t OOB = 0x80000000u; // buffer offset past every range: load 0, store dropped
constexpr int AUX_NT = 2;             // buffer cache policy: nontemporal (the streaming loads)
// Policy of the payload stores: nontemporal (the run decoder); the lattice
// decoder's streaming stores are sc1 | nt, written through past
// the XCD's L2 (a decode never reads its stores back): c3 0.6712 -> 0.6512
// ms, c1 0.1106 -> 0.1090 against nt alone, same box; sc1 alone 0.6564,
// plain 0.7198 (profiles/r05y_store_policy_ab.txt); the run decoder measured
// 0.5126 vs 0.5015 ms on c4 with them (r05z vs r05x) and keeps nt
#ifndef XYWS_EXP_AUX_ST
#define XYWS_EXP_AUX_ST 2
#endif
constexpr int AUX_ST = XYWS_EXP_AUX_ST;
constexpr int AUX_ST_STREAM = 18;
constexpr uint64_t PLEN_SPEC_MAX = 1ull << 46;
constexpr uint32_t MAX_RUNS = 1024;
// work stealing: a run is asked for its tail when it has at least this many
// segments left after the current one; the piece is at least this long
#ifndef XYWS_STEAL_MIN_LEFT
#define XYWS_STEAL_MIN_LEFT 8
#endif
#ifndef XYWS_STEAL_MIN_PIECE
#define XYWS_STEAL_MIN_PIECE 3
#endif


// chase-state bits
constexpr uint32_t S_PARTIAL = 1;    // header at X incomplete at the batch end
constexpr uint32_t S_NOCOV = 2;      // no frame covers the bytes before X
constexpr uint32_t S_CARRIED = 4;    // covering frame = the open frame carried in
constexpr uint32_t S_HDRCARRY = 8;   // covering frame's header began in the previous batch
constexpr uint32_t S_PARTCARRY = 16; // the carried partial header is still incomplete
constexpr uint32_t S_CUT = 32;       // header at X crosses the write limit (left to the repair)

template <uint32_t NT_, uint32_t CH_, uint32_t WPE_>
struct geom {
  // threads, 16-byte chunks per thread, waves per SIMD the decode kernel must
  // fit (register budget 512 / WPE)
  static constexpr uint32_t NT = NT_, CH = CH_, SEG = NT_ * CH_ * 16, WPE = WPE_;
  static constexpr uint32_t SEGX = SEG;  // (bytes of the segment readable from LDS)
  // frame-list entries per pass (one per thread: the dense pass compacts them
  // one per thread); prologue lists overlaying the frame list
  static constexpr uint32_t FCAP = NT_, SCAP = NT_ * 2, UCAP = NT_ * 2;
  // dense pass: sub-blocks (entries: 16 lanes each), their bytes and list sections
  static constexpr uint32_t NSB = NT_ / 16, SB = SEG / NSB, SECT = FCAP / NSB;
};
using G_PROD = geom<1024, 8, 4>;  // 128 KiB segments, 16 waves, one workgroup per CU (default)
using G_PROD2 = geom<512, 8, 4>;  // 64 KiB segments, 8 waves, two workgroups per CU (XYWS_OPT_WG512)
using G_SMALL = geom<64, 1, 1>;   // 1 KiB segments, one wave (XYWS_OPT_SMALL_SEG)
using G_MID = geom<256, 4, 4>;    // 16 KiB segments, 4 waves, four workgroups per CU (mid_preferred)

struct fent {
  uint32_t start, ps, end, kw;  // segment-relative, clamped to [0, 2^32-1]
};

struct cstate {
  uint64_t X;          // next frame start (absolute)
  uint64_t cov_ps;     // payload start of the frame covering the bytes before X
  uint64_t cov_start;  // its header start
  uint32_t cov_kw;     // its aligned key word
  uint32_t cov_key;    // its key (wire order)
  uint32_t st;         // S_* bits
  uint32_t pad;
};

// finish_walk: the current chain piece (see the walk below).
struct walk_t {
  cstate F;
  uint64_t r, efrom, cnt, tail, first, succ, wlim;
  uint32_t ok, tmo, ecarry, act;
};

// run record: R_WORDS x u64
enum {
  R_H = 0, R_W, R_S0, R_HEAD = R_S0 + 5,            // prologue: entry, write start, state, head frames
  R_OK = 8, R_HN, R_WN, R_CNT, R_TAIL, R_FIRST,     // results (R_OK: ok | tmo << 1 | succ << 32)
  R_F0 = 14,                                        // final state (5 words)
  R_EFROM = 20, R_ECNT, R_EORD, R_ECARRY,           // emission plan (finish_call)
  R_EP = 24,                                        // epoch of the call that wrote the results
  R_T0, R_T1, R_T2,                                 // stats mode: s_memrealtime at start, after the prologue, at the end
  R_SPLIT,                                          // own runs: the split segment a thief took the rest from (NONE: none)
  R_XCC,                                            // stats mode: the XCD (XCC_ID) the run's workgroup ran on
  R_NREC,                                           // descriptors requested: frame starts in the item's region
  R_WORDS = 32
};
// R_OK bits
constexpr uint64_t OK_BIT = 1, TMO_BIT = 2;  // chain landed on the successor; successor wait timed out

// Entry granules, 16 bytes per run, each written by ONE 16-byte sc1 store and
// read by ONE 16-byte sc1 load (MI355X_MICROARCH.md §inter-workgroup
// visibility: 16-B granules observed untorn), stamped with the call's epoch E
// (head word HEAD_EPOCH holds the number of completed calls; a call runs with
// E = that + 1):
//   word 0: (E << 1) = claimed by the run's own workgroup in this call,
//           (E << 1) | 1 = published; anything below E << 1 is a previous
//           call's and reads as unclaimed (no per-call reset, no stale record);
//   word 1 (published): h (46 bits, G_NONE = no entry) | (W - h) << 46 (5
//           bits: W = round16(h + header)) | (E mod 2^13) << 51, the tag a
//           torn read would fail.
// The run's record (R_H, R_W, entry state, ...) is for finish_call only,
// so the publish needs no wait for the record stores (nor for the prefetch
// loads in flight).
XYWS_DEV uint64_t flag_claimed(uint64_t E) { return E << 1; }
XYWS_DEV uint64_t flag_published(uint64_t E) { return (E << 1) | 1u; }
constexpr uint64_t G_NONE = (1ull << 46) - 1;
XYWS_DEV uint64_t granule_tag(uint64_t E) { return (E & 0x1FFFull) << 51; }
constexpr uint32_t HEAD_EPOCH = 4;   // u32 index of the u64 epoch word in head[]
// End-of-call words (u64 indices in head[], bytes 512..576), zeroed at
// allocation and reset by the workgroup that finishes the call: workgroups
// done, hand-overs that need the repair walk, frames of all items, and the
// final chain state of the item whose chain reached the batch end.
constexpr uint32_t HW_DONE = 64, HW_BAD = 65, HW_TOTAL = 66, HW_FINAL = 67;
// descriptor emission: non-zero when the frame-start lists cannot be used (a
// region overflowed, or a repaired hand-over changed the plan) and
// k_stream_emit re-walks the chains instead
constexpr uint32_t HW_EMIT_SLOW = 73;
// ...copied by finish_call for k_stream_emit (and reset there)
constexpr uint32_t HW_EMIT_FLAG = 74;
// decoder choice (stream_decode_fused): the largest and (complemented) the
// smallest size of the last frame of every run / segment exit of the call,
// published by the finisher into the context's host-visible policy slot
constexpr uint32_t HW_FSMAX = 75, HW_FSMIN = 76;

XYWS_DEV void granule_store(uint64_t* g, uint64_t a, uint64_t b) {
  const u32x4 v = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(g), "v"(v) : "memory");
}
XYWS_DEV void granule_load(const uint64_t* g, uint64_t& a, uint64_t& b) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(g) : "memory");
  a = (uint64_t)v.x | ((uint64_t)v.y << 32);
  b = (uint64_t)v.z | ((uint64_t)v.w << 32);
}

// Work stealing. A run's range is cut at segment granularity when a workgroup
// that finished early asks for it: the tail of the range becomes a PIECE that
// the thief decodes like a run (its own entry scan, chain and record), placed
// between the run and its successor. Records, entry granules and descriptor
// plans are indexed by a flat index in batch order: run r = 2r, its piece =
// 2r + 1 (at most one piece per run). Per run, a split word (16 bytes, the
// first u64 used) holds (E << 24) | (state << 22) | e', e' the first segment
// of the piece:
//   FREE   set by the run when it starts (it can be asked),
//   REQ    a thief asks (atomic CAS from FREE),
//   ACC    the run agrees, the piece starts at segment e',
//   CLS    the run will not split (no entry, too little left, successor
//          already looked up, or a refused request).
// The run reads its split word with one load per segment (lane 0, issued
// before the prefetch and used one iteration later: no stall).
enum { SP_FREE = 0, SP_REQ = 1, SP_ACC = 2, SP_CLS = 3 };
XYWS_DEV uint64_t split_word(uint64_t E, uint32_t state, uint32_t e) {
  return (E << 24) | ((uint64_t)state << 22) | (e & 0x3FFFFFu);
}
XYWS_DEV uint32_t split_state(uint64_t w) { return (uint32_t)(w >> 22) & 3u; }
XYWS_DEV uint32_t split_seg(uint64_t w) { return (uint32_t)w & 0x3FFFFFu; }
XYWS_DEV bool split_is(uint64_t w, uint64_t E, uint32_t state) { return (w >> 24) == (E & ((1ull << 40) - 1)) && split_state(w) == state; }

struct run_params {
  uint8_t* base;
  uint64_t lo, hi;
  uint64_t rbytes;        // bytes per run range (multiple of 16); run r: [r*rbytes, (r+1)*rbytes)
  uint32_t nruns;
  uint32_t nflat;         // 2 * nruns: records / granules / plans (run r = 2r, its piece = 2r + 1)
  uint64_t* split;        // per run: split word (2 x u64)
  uint64_t* prog;         // per run: (E << 24) | segment being decoded (thieves pick the run with most left)
  const xyws_carry* cin_user;  // caller's incoming carry (nullable; may alias cout)
  uint64_t pfs;                // run decoder: the frame size the previous call's frames all had (0: none;
                               // find_entry's lattice entry)
  uint32_t dense0;             // run decoder: the previous call's frames were small and of mixed sizes:
                               // a run's first segment goes to the dense pass at once (no stride try)
  uint32_t bigscan;            // entry scans: the previous call's frames had mixed sizes, some large
                               // (find_entry: no window-0 pass, undecided chains carried forward)
  xyws_carry* cin;        // private snapshot of it, written by run 0 (finish/emit read it)
  xyws_carry* cout;
  xyws_frame* frames;
  uint64_t cap;
  uint64_t* nframes;
  uint64_t* rec;          // R_WORDS per flat index
  uint64_t* flags;        // per flat index: entry granule (2 x u64, see flag_claimed)
  uint32_t* head;         // [0] ticket, [1] error word, [2..3] u64 total, [4..5] u64 epoch;
                          // [16..32) carry snapshot; stats at [32..)
  uint32_t opts;
  // descriptors requested: the starts of the frames each item (run or piece)
  // finds, in chain order, in its own region of rcap entries (fst + item *
  // rcap); k_stream_emit writes the descriptors from them in parallel
  uint64_t* fst;
  uint64_t rcap;
  uint64_t nseg;  // lattice decoder: segments of the batch
  // host-visible policy slot (device address of pinned host memory; nullable):
  // written by the workgroup that finishes the call (pol_publish)
  uint64_t* pol;
  // lattice decoder (xyws_lattice.h): its scratch words (claims, epoch,
  // per-segment results, the redirect record the run decoder reads with
  // XYWS_OPT_REDIRECT); the run decoder's segment size (lat_redirect cuts
  // the rest of a batch into runs with it); frames decoded before a
  // redirected batch (counts and ordinals go on from there) and the offset of
  // its start in the caller's batch (descriptor offsets)
  uint64_t* lat;
  uint64_t* lgrp;  // lattice decoder: decided-segment counts per LAT_GRP segments
  uint64_t* lbrk;  // lattice decoder: the replicas of LW_BRK
  uint64_t* lsl;   // lattice decoder: the workgroups' speculative-store lists (LAT_LSW words each)
  uint32_t segb;
  uint64_t tbias, obias;
};

// (xyws_lattice.h, included below)
XYWS_DEV bool lat_redirect(run_params& P);

template <class G>
struct __attribute__((aligned(16))) lds_t {
  uint8_t seg[G::SEG + PAD];
  union {
    fent fl[G::FCAP];
    struct {  // prologue: survivors of a segment's scan filter, and those whose chain left the segment
      uint32_t sl[G::SCAP];
      uint32_t ul[G::UCAP];
    };
  };
  cstate S;
  cstate B;  // finish_call: exact state handed to a repaired run
  uint64_t hn, Wn, succ, first_after, cnt, tail, aux0, aux1, aux2, bcnt, bfirst;
  uint64_t E;      // this call's epoch
  xyws_carry cinc; // finish_call: the incoming-carry snapshot
  uint64_t scan_j; // successor lookup: next flat index to examine
  uint64_t ib, ie;     // the item (own run or piece) the workgroup decodes next: its byte range
  uint64_t rng_end;    // end of the current run's range (a run's shrinks when a thief takes its tail)
  uint64_t rs;         // start of the current run's range (segment grid of the split word)
  uint64_t split_e;    // own run: first segment of the piece taken from it (NONE: none)
  uint64_t split_poll[2] __attribute__((aligned(16)));  // the run's split word at the start of an item
  uint64_t self;       // flat index of the run or piece being decoded
  uint32_t victim;     // 1: the current run answers steal requests (an own run, not yet closed)
  walk_t wk;       // finish_call: the current chain piece
  uint32_t nfl, pass_hi, known, past, ok, done, end, best, ticket, act, repaired, ccnt, ucnt, keepn, ovf;
  uint32_t tmo;    // successor given up on (write limit = own range end, bridged by finish_call)
  // per 1 KiB row of the segment (one wave-instruction of chunks), set by
  // wave 0 after each chase pass: ROW_FAST (one key word for the whole row,
  // rk), ROW_SKIP (nothing to store) or the entry to start the walk from
  uint2 rt[G::SEG / 1024];  // (class or entry, key word)
  // dense pass, per sub-block: speculated entry, frames, exit, last frame
  // (start, payload start, key, key word)
  uint32_t dent[G::NSB], dcnt[G::NSB], dexit[G::NSB], doff[G::NSB];
  uint4 dlast[G::NSB];
  uint32_t dense;  // frames of the previous pass (the dense pass is tried after a dense one)
  uint32_t sgood;  // the stride pass serves dense segments (cleared when it did not cover one)
  // lattice pass (run_chain): entries 1.. start at ar_x0 + (i - 1) * ar_f
  uint32_t ar, ar_x0, ar_f;
  uint32_t nrec;   // descriptors requested: frame starts the current item recorded
};

// ---------------------------------------------------------------- small helpers
XYWS_DEV void st_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
XYWS_DEV uint64_t st_load(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
XYWS_DEV bool stats_on(const run_params& P) { return (P.opts & XYWS_OPT_STATS) != 0; }
enum { ST_RUNS = 0, ST_NONE, ST_BAD, ST_REPAIR, ST_CUT, ST_SPIN, ST_SEGS, ST_FRAMES,
       ST_P_WIN, ST_P_CAND, ST_P_UND, ST_P_TCOMP, ST_P_TCHECK, ST_P_TRES, ST_D_TENT, ST_D_TCHASE,
       ST_T_PRO = 16, ST_T_MAIN, ST_T_WAIT, ST_T_FILL, ST_T_CHASE, ST_T_XOR, ST_T_TAIL, ST_T_PF, ST_T_CP,
       ST_P_FILL, ST_P_SCAN, ST_P_PUB, ST_D_NOENT, ST_D_CHASE, ST_D_MISMATCH, ST_D_OVF,
       ST_GIVEUP = 32, ST_BRIDGE, ST_STEAL_REQ, ST_STEAL_ACC, ST_STEAL_SEGS, ST_D_TVAL, ST_T_ROWS, ST_T_SER,
       ST_X_W0 = 41, ST_X_BITS = 42, ST_X_SURV = 43,  // entry scan (lane 0): window 0 to its check; the
                            // rest's candidate bits (from the segment's start); its survivors loop
       ST_T_STRIDE = 46,    // the run decoder's stride-pass time
       ST_P_LATTICE = 40 }; // runs whose entry the lattice gave
XYWS_DEV void stat_add(const run_params& P, uint32_t i, uint64_t v) {
  if (stats_on(P)) atomicAdd(reinterpret_cast<unsigned long long*>(P.head + 32) + i, (unsigned long long)v);
}

// The size of the frame a chain state last completed (H + P), for the
// decoder choice: 0 when the state holds no whole frame of this batch.
XYWS_DEV uint64_t last_frame_size(const cstate& S);
// Lane 0 of a run or segment: fold a last-frame size into the call's min/max.
XYWS_DEV void fs_note(const run_params& P, uint64_t fsmin, uint64_t fsmax) {
  uint64_t* hw = reinterpret_cast<uint64_t*>(P.head);
  if (!fsmax) return;
  __hip_atomic_fetch_max(hw + HW_FSMAX, fsmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_max(hw + HW_FSMIN, ~fsmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The device-resident copy of the decoder-choice words, written by the
// workgroup finishing a call: bit 63 a call has finished, bits 48..55 its
// decoder, bits 0..47 the size every last frame of the call had (0: mixed
// sizes). In the run scratch's head (u64 HW_DPOL, zeroed at allocation) and
// in the lattice scratch when the context has one (LW_DPOL, next to the
// lattice epoch: xyws_lattice.h). The lattice decoder's prologue loads it
// with its epoch, so its first-segment gate and its bail-out after an
// irregular call follow the previous call in the stream, not the host's view
// of the pinned words (which lags by the calls in flight).
enum : uint64_t { DEC_RUNS = 0, DEC_RUNS512 = 2, DEC_LATTICE = 3 };
constexpr uint32_t HW_DPOL = 77;
constexpr uint32_t LW_DPOL_WORD = 6;  // (= LW_DPOL, xyws_lattice.h)
XYWS_DEV void dpol_publish(const run_params& P, uint64_t F, uint64_t decoder) {
  const uint64_t f = F < (1ull << 48) ? F : 0;
  const uint64_t v = (1ull << 63) | (decoder << 48) | f;
  st_store(reinterpret_cast<uint64_t*>(P.head) + HW_DPOL, v);
  if (P.lat) st_store(P.lat + LW_DPOL_WORD, v);
}
// The finisher (lane 0): the call's frame-size range into the host-visible
// policy slot {epoch, batch bytes, smallest, largest last-frame size, decoder}
// (and its device copy) and the words reset for the next call. Host memory:
// system-scope stores.
XYWS_DEV void pol_publish(const run_params& P, uint64_t E, uint64_t decoder) {
  uint64_t* hw = reinterpret_cast<uint64_t*>(P.head);
  const uint64_t mx = st_load(hw + HW_FSMAX), mn = ~st_load(hw + HW_FSMIN);
  st_store(hw + HW_FSMAX, 0);
  st_store(hw + HW_FSMIN, 0);
  dpol_publish(P, mx && mn == mx ? mx : 0, decoder);
  if (!P.pol) return;
  const uint64_t v[5] = {E, P.hi - P.lo, mx ? mn : 0, mx, decoder};
#pragma unroll
  for (int i = 1; i < 5; i++) __hip_atomic_store(P.pol + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(P.pol, v[0], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

XYWS_DEV uint32_t clamp_rel(uint64_t x, uint64_t ss) {
  if (x <= ss) return 0;
  const uint64_t d = x - ss;
  return d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
}

XYWS_DEV void put_state(uint64_t* r, const cstate& s) {
  st_store(r + 0, s.X);
  st_store(r + 1, s.cov_ps);
  st_store(r + 2, s.cov_start);
  st_store(r + 3, (uint64_t)s.cov_kw | ((uint64_t)s.cov_key << 32));
  st_store(r + 4, s.st);
}
XYWS_DEV cstate get_state(const uint64_t* r) {
  cstate s;
  s.X = st_load(r + 0);
  s.cov_ps = st_load(r + 1);
  s.cov_start = st_load(r + 2);
  const uint64_t k = st_load(r + 3);
  s.cov_kw = (uint32_t)k;
  s.cov_key = (uint32_t)(k >> 32);
  s.st = (uint32_t)st_load(r + 4);
  s.pad = 0;
  return s;
}
XYWS_DEV cstate frame_state(uint64_t start, const hdr_info& h) {
  cstate s;
  s.cov_start = start;
  s.cov_ps = start + h.hlen;
  s.X = sat_add(s.cov_ps, h.plen);
  s.cov_key = h.key;
  s.cov_kw = aligned_key(h.key, s.cov_ps, 0);
  s.st = 0;
  s.pad = 0;
  return s;
}

XYWS_DEV uint64_t last_frame_size(const cstate& S) {
  const bool whole = !(S.st & (S_NOCOV | S_PARTIAL | S_PARTCARRY | S_CARRIED | S_HDRCARRY | S_CUT));
  return (whole && S.X > S.cov_start && S.X != ~0ull) ? S.X - S.cov_start : 0;
}

// ---------------------------------------------------------------- header reads
// Header at absolute x from memory, using only bytes below lim (and hi).
XYWS_DEV hdr_info hdr_global(const run_params& P, uint64_t x, uint64_t lim) {
  hdr_info h;
  h.plen = 0; h.key = 0; h.hlen = 0; h.flags = 0; h.status = 0;
  const uint64_t top = lim < P.hi ? lim : P.hi;
  if (x >= top) return h;
  const uint64_t a = x & ~3ull;
  const uint32_t sh = (uint32_t)(x & 3);
  const uint64_t dl = (P.hi + 3) & ~3ull;  // dwords wholly or partly inside the batch
  uint32_t r[5];
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint64_t q = a + 4 * i;
    r[i] = q < dl ? *reinterpret_cast<const uint32_t*>(P.base + q) : 0u;
  }
  // wait here (vmcnt 0, other counters untouched) so that no register leaves
  // this branch with a load pending: otherwise the compiler's wait lands after
  // the join with the LDS path and every header parse waits for the segment
  // prefetch in flight
  __builtin_amdgcn_s_waitcnt(0x0F70);
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
  const uint64_t room = top - x;
  return parse_header_words(w, room < 16 ? (uint32_t)room : 16u);
}

// Header at absolute x: from the LDS copy of segment [ss, ss+SEG) when all 14
// possible bytes lie in it, else from memory.
template <class G>
XYWS_DEV hdr_info hdr_at(const run_params& P, const lds_t<G>& L, uint64_t ss, uint64_t x, uint64_t lim) {
  const uint64_t top = lim < P.hi ? lim : P.hi;
  if (x >= ss && x - ss + XYWS_MAX_FRAME_HEADER_SIZE <= G::SEGX && x < top) {
    const uint32_t o = (uint32_t)(x - ss), a = o & ~3u, sh = o & 3u;
    const uint32_t* q = reinterpret_cast<const uint32_t*>(L.seg + a);
    const uint32_t r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
    uint32_t w[4];
    w[0] = __builtin_amdgcn_alignbyte(r1, r0, sh);
    w[1] = __builtin_amdgcn_alignbyte(r2, r1, sh);
    w[2] = __builtin_amdgcn_alignbyte(r3, r2, sh);
    w[3] = __builtin_amdgcn_alignbyte(r4, r3, sh);
    const uint64_t room = top - x;
    return parse_header_words(w, room < 16 ? (uint32_t)room : 16u);
  }
  return hdr_global(P, x, lim);
}

// Header whose first h0 bytes were carried from the previous batch (the rest
// from the batch start), assembled in registers.
XYWS_DEV hdr_info header_carried(const run_params& P, const xyws_carry* c) {
  const uint32_t h0 = c->hdr_len < XYWS_MAX_FRAME_HEADER_SIZE ? c->hdr_len : XYWS_MAX_FRAME_HEADER_SIZE;
  uint32_t w[4] = {0u, 0u, 0u, 0u}, n = 0;
#pragma unroll
  for (uint32_t i = 0; i < XYWS_MAX_FRAME_HEADER_SIZE; i++) {
    uint32_t b = 0;
    bool have = true;
    if (i < h0) b = c->hdr[i];
    else if (P.lo + (i - h0) < P.hi) b = P.base[P.lo + (i - h0)];
    else have = false;
    if (have && n == i) {
      w[i >> 2] |= b << (8u * (i & 3u));
      n++;
    }
  }
  return parse_header_words(w, n);
}

// A header a client stream plausibly holds (speculation only).
XYWS_DEV bool plausible(const hdr_info& h, bool unmasked) {
  if (!h.hlen) return false;
  if (h.status & (XYWS_ST_RSV | XYWS_ST_RESERVED_OPCODE | XYWS_ST_NONMINIMAL_LENGTH |
                  XYWS_ST_LENGTH_MSB | XYWS_ST_BAD_CONTROL))
    return false;
  if (((h.status & XYWS_ST_UNMASKED) != 0) != unmasked) return false;
  return h.plen < PLEN_SPEC_MAX;
}

// Four candidate bits (bytes 0..3 of w) for a client header: RSV = 0, opcode in
// {0,1,2} or {8,9,10} with FIN, MASK bit (first bit of the next byte) as
// expected. A superset of plausible().
XYWS_DEV uint32_t cand_nibble(uint32_t w, uint32_t wn, bool unmasked) {
  const uint32_t b1s = (w >> 8) | (wn << 24);  // byte t = byte t+1
  const uint32_t rsv_ok = ~((w & 0x70707070u) + 0x70707070u) & 0x80808080u;
  const uint32_t bad = ((w << 5) | ((w << 6) & (w << 7)) | ((w << 4) & ~w)) & 0x80808080u;
  const uint32_t m_ok = (unmasked ? ~b1s : b1s) & 0x80808080u;
  const uint32_t c = rsv_ok & ~bad & m_ok;
  return ((c >> 7) & 1u) | ((c >> 14) & 2u) | ((c >> 21) & 4u) | ((c >> 28) & 8u);
}

// Candidate bits of the 16 positions of chunk a (bit t: position a + t).
template <class G>
XYWS_DEV uint32_t chunk_candidates(const run_params& P, const lds_t<G>& L, uint32_t a, bool unm) {
  const u32x4 v = *reinterpret_cast<const u32x4*>(L.seg + a);
  const uint32_t w4 = *reinterpret_cast<const uint32_t*>(L.seg + a + 16);
  uint32_t bits = cand_nibble(v.x, v.y, unm) | (cand_nibble(v.y, v.z, unm) << 4) |
                  (cand_nibble(v.z, v.w, unm) << 8) | (cand_nibble(v.w, w4, unm) << 12);
  // headers straddling the segment end are left to the next segment's scan
  if (a + 16 + 1 > G::SEG) bits &= (1u << (G::SEG - XYWS_MAX_FRAME_HEADER_SIZE - a + 1)) - 1u;
  return bits;
}

// Candidate bits of the 4 positions of dword w (wn: the next dword) at bits
// 7, 15, 23, 31: the cand_nibble test with fewer operations.
XYWS_DEV uint32_t cand_bytes(uint32_t w, uint32_t wn, bool unmasked) {
  const uint32_t b1s = __builtin_amdgcn_alignbyte(wn, w, 1);               // byte t = byte t+1
  const uint32_t rsv = ((w & 0x74747474u) + 0x7F7F7F7Fu);                    // RSV or opcode bit 2
  const uint32_t b3 = (w << 7) & (w << 6);                                   // opcode & 3 == 3
  const uint32_t ctl = (w << 4) & ~w;                                        // control without FIN
  const uint32_t m = unmasked ? ~b1s : b1s;
  return m & ~(rsv | b3 | ctl) & 0x80808080u;
}

// First byte pair of a client header (cand_nibble for one position).
XYWS_DEV bool cand_pair(uint32_t b0, uint32_t b1, bool unm) {
  return (b0 & 0x74u) == 0 && (b0 & 3u) != 3u && !((b0 & 0x08u) && !(b0 & 0x80u)) &&
         ((b1 >> 7) != 0) != unm;
}

// The carry as its 8 words in registers (xyws_carry: payload_remaining,
// phase, frames_total, key[4] @24, hdr_len @28, hdr[14] @29): byte k by
// shifts of constant amounts once unrolled, so no copy of the struct is
// placed in scratch (the lattice decoder's prologue loads the words at once).
struct carry_words {
  uint64_t w[8];
  XYWS_DEV uint32_t byte(uint32_t k) const { return (uint32_t)(w[k >> 3] >> (8u * (k & 7u))) & 0xFFu; }
};
XYWS_DEV cstate initial_state_w(const run_params& P, const carry_words& c, uint64_t& cnt) {
  cstate s;
  s.X = P.lo; s.cov_ps = P.lo; s.cov_start = P.lo; s.cov_kw = 0; s.cov_key = 0; s.st = S_NOCOV; s.pad = 0;
  cnt = 0;
  const uint64_t R = c.w[0];
  if (R) {
    const uint32_t k = (uint32_t)c.w[3];
    s.X = sat_add(P.lo, R);
    s.cov_kw = aligned_key(k, P.lo, c.w[1]);
    s.cov_key = k;
    s.st = S_CARRIED;
    return s;
  }
  const uint32_t hl = c.byte(28);
  if (hl) {
    const uint32_t h0 = hl < XYWS_MAX_FRAME_HEADER_SIZE ? hl : XYWS_MAX_FRAME_HEADER_SIZE;
    uint32_t w[4] = {0u, 0u, 0u, 0u}, n = 0;
#pragma unroll
    for (uint32_t i = 0; i < XYWS_MAX_FRAME_HEADER_SIZE; i++) {
      uint32_t b = 0;
      bool have = true;
      if (i < h0) b = c.byte(29 + i);
      else if (P.lo + (i - h0) < P.hi) b = P.base[P.lo + (i - h0)];
      else have = false;
      if (have && n == i) {
        w[i >> 2] |= b << (8u * (i & 3u));
        n++;
      }
    }
    const hdr_info h = parse_header_words(w, n);
    if (!h.hlen) {  // still incomplete: the whole batch belongs to the header
      s.st = S_NOCOV | S_PARTIAL | S_PARTCARRY;
      return s;
    }
    s = frame_state(P.lo, h);
    s.cov_ps = P.lo + (h.hlen - hl);
    s.X = sat_add(s.cov_ps, h.plen);
    s.cov_kw = aligned_key(h.key, s.cov_ps, 0);
    s.st = S_HDRCARRY;
    cnt = 1;
  }
  return s;
}

// State before the first byte of the batch, from the carry snapshot; cnt =
// frames it completes (the carried-header frame).
XYWS_DEV cstate initial_state(const run_params& P, const xyws_carry* c, uint64_t& cnt) {
  cstate s;
  s.X = P.lo; s.cov_ps = P.lo; s.cov_start = P.lo; s.cov_kw = 0; s.cov_key = 0; s.st = S_NOCOV; s.pad = 0;
  cnt = 0;
  const uint64_t R = c->payload_remaining;
  if (R) {
    const uint32_t k = (uint32_t)c->key[0] | ((uint32_t)c->key[1] << 8) |
                       ((uint32_t)c->key[2] << 16) | ((uint32_t)c->key[3] << 24);
    s.X = sat_add(P.lo, R);
    s.cov_kw = aligned_key(k, P.lo, c->phase);
    s.cov_key = k;
    s.st = S_CARRIED;
    return s;
  }
  if (c->hdr_len) {
    const hdr_info h = header_carried(P, c);
    if (!h.hlen) {  // still incomplete: the whole batch belongs to the header
      s.st = S_NOCOV | S_PARTIAL | S_PARTCARRY;
      return s;
    }
    s = frame_state(P.lo, h);
    s.cov_ps = P.lo + (h.hlen - c->hdr_len);
    s.X = sat_add(s.cov_ps, h.plen);
    s.cov_kw = aligned_key(h.key, s.cov_ps, 0);
    s.st = S_HDRCARRY;
    cnt = 1;
  }
  return s;
}

// ---------------------------------------------------------------- segment I/O
template <class G>
XYWS_DEV __amdgpu_buffer_rsrc_t seg_rsrc(const run_params& P, uint64_t ss, uint64_t lim = NONE) {
  // [ss, ss + min(SEG, top - ss)), top = min(round16(hi), lim): loads past it
  // read zero without touching memory
  uint64_t top = (P.hi + 15) & ~15ull;
  if (lim < top) top = (lim + 15) & ~15ull;
  const uint64_t room = top > ss ? top - ss : 0;
  const uint32_t n = room >= G::SEG ? G::SEG : (uint32_t)room;
  return __builtin_amdgcn_make_buffer_rsrc(P.base + ss, 0, n, 0x00020000);
}

template <class G>
struct seg_io {
  u32x4 e[G::CH];
  uint64_t pf = NONE;  // start of the segment whose loads are in e
  // loads of the segment at ss (bytes at or past lim are not needed: zero)
  XYWS_DEV void issue(const run_params& P, uint64_t ss, uint32_t tid, uint64_t lim = NONE) {
    const __amdgpu_buffer_rsrc_t rs = seg_rsrc<G>(P, ss, lim);
#pragma unroll
    for (uint32_t k = 0; k < G::CH; k++)
      e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16u, k * G::NT * 16u, AUX_NT);
    pf = ss;
  }
  // the segment at ss into LDS (caller syncs before and after)
  XYWS_DEV void fill(const run_params& P, lds_t<G>& L, uint64_t ss, uint32_t tid) {
    if (pf != ss) issue(P, ss, tid);
#pragma unroll
    for (uint32_t k = 0; k < G::CH; k++)
      *reinterpret_cast<u32x4*>(&L.seg[(k * G::NT + tid) * 16u]) = e[k];
    pf = NONE;
  }
};

// ---------------------------------------------------------------- the chase
// XOR words for the 16-byte chunk at segment offset a; entries are contiguous
// frames sorted by start, g = the last entry starting at or before a.

// The key word kw on the bytes of the 16-byte chunk at a that lie in [lo, hi)
// (segment-relative, any values): the byte mask as two 64-bit halves from the
// clamped chunk-relative bounds (a few shifts, no per-dword range tests).
XYWS_DEV u32x4 span_key16(uint32_t a, uint32_t lo, uint32_t hi, uint32_t kw) {
  const uint32_t l = lo <= a ? 0u : lo - a >= 16u ? 16u : lo - a;
  const uint32_t h = hi <= a ? 0u : hi - a >= 16u ? 16u : hi - a;
  const uint64_t one = ~0ull;
  // bytes [0, h) and [0, l) of the chunk, each as (low half, high half)
  const uint64_t h0 = h >= 8 ? one : ~(one << (8u * h)), h1 = h >= 16 ? one : h > 8 ? ~(one << (8u * (h - 8))) : 0ull;
  const uint64_t l0 = l >= 8 ? one : ~(one << (8u * l)), l1 = l >= 16 ? one : l > 8 ? ~(one << (8u * (l - 8))) : 0ull;
  const uint64_t k = (uint64_t)kw | ((uint64_t)kw << 32);
  const uint64_t m0 = (h0 & ~l0) & k, m1 = (h1 & ~l1) & k;
  return u32x4{(uint32_t)m0, (uint32_t)(m0 >> 32), (uint32_t)m1, (uint32_t)(m1 >> 32)};
}

XYWS_DEV u32x4 chunk_xor(const fent* fl, uint32_t nfl, uint32_t g, uint32_t a) {
  u32x4 w = {0u, 0u, 0u, 0u};
  for (uint32_t h = g; h < nfl; h++) {
    const fent f = fl[h];
    if (h != g && f.start >= a + 16) break;
    w |= span_key16(a, f.ps, f.end, f.kw);
  }
  return w;
}

// 32-bit parse of the header at segment offset x whose 14 bytes are in LDS:
// header length, payload length, key (wire order) and the first two bytes.
// False for a payload length of 2^31 or more (left to the 64-bit parse).
template <class G>
XYWS_DEV bool parse_rel(const lds_t<G>& L, uint32_t x, uint32_t& hl, uint32_t& plen, uint32_t& key, uint32_t& b01) {
  // (no branches: the three length forms and key positions are selected, so
  // a chase step is one straight run of instructions after its LDS reads)
  const uint32_t* q = reinterpret_cast<const uint32_t*>(L.seg + (x & ~3u));
  const uint32_t sh = x & 3u, r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
  const uint32_t w0 = __builtin_amdgcn_alignbyte(r1, r0, sh), w1 = __builtin_amdgcn_alignbyte(r2, r1, sh);
  const uint32_t w2 = __builtin_amdgcn_alignbyte(r3, r2, sh), w3 = __builtin_amdgcn_alignbyte(r4, r3, sh);
  b01 = w0 & 0xFFFFu;
  const uint32_t l7 = (w0 >> 8) & 0x7Fu, msk = (w0 >> 15) & 1u;
  const bool s7 = l7 < 126, s16 = l7 == 126;
  const uint32_t hi32 = __builtin_amdgcn_alignbyte(w1, w0, 2);  // bytes 2..5
  const uint32_t lo32 = __builtin_amdgcn_alignbyte(w2, w1, 2);  // bytes 6..9
  const uint32_t p16 = ((w0 >> 8) & 0xFF00u) | (w0 >> 24);
  plen = s7 ? l7 : (s16 ? p16 : __builtin_bswap32(lo32));
  hl = 2u + (s7 ? 0u : (s16 ? 2u : 8u)) + 4u * msk;
  const uint32_t k = s7 ? hi32 : (s16 ? w1 : __builtin_amdgcn_alignbyte(w3, w2, 2));
  key = msk ? k : 0u;
  return s7 || s16 || (hi32 == 0u && !(lo32 & 0x80u));  // lengths >= 2^31: the general step
}

// Descriptors requested (lane 0): the k frames starting at frame-list entry
// `first` (segment-relative starts), the item's own frames found by this pass,
// appended to the item's region. An overflow switches the emission to the
// chain re-walk.
XYWS_DEV void flag_emit_slow(const run_params& P) {
  __hip_atomic_fetch_or(reinterpret_cast<uint64_t*>(P.head) + HW_EMIT_SLOW, 1ull, __ATOMIC_RELAXED,
                        __HIP_MEMORY_SCOPE_AGENT);
}
template <class G>
XYWS_DEV void record_starts(const run_params& P, lds_t<G>& L, uint64_t ss, uint32_t first, uint32_t k) {
  if (!P.fst || !k) return;
  const uint64_t n = L.nrec;
  if (n + k > P.rcap) { flag_emit_slow(P); return; }
  uint64_t* dst = P.fst + L.self * P.rcap + n;
#pragma unroll 1
  for (uint32_t i = 0; i < k; i++) dst[i] = ss + L.fl[first + i].start;
  L.nrec = (uint32_t)(n + k);
}
// one frame start (absolute): the prologue's head frames
template <class G>
XYWS_DEV void record_start(const run_params& P, lds_t<G>& L, uint64_t self, uint64_t x) {
  if (!P.fst) return;
  if (L.nrec + 1 > P.rcap) { flag_emit_slow(P); return; }
  P.fst[self * P.rcap + L.nrec] = x;
  L.nrec++;
}

// An all-zero carry (a decode without incoming carry).
__device__ const xyws_carry k_zero_carry = {};

// One pass of the chase over segment [ss, ss+SEG), lane 0: the frame covering
// the pass start, then frames parsed from X, up to G::FCAP entries. Sets
// pass_hi: the chunks below it are final for this pass.
template <class G>
XYWS_DEV void chase_pass(const run_params& P, lds_t<G>& L, uint64_t ss, uint32_t lo_c, uint32_t keep) {
  const uint64_t se = ss + G::SEG;
  cstate S = L.S;
  uint32_t n = keep;  // entries carried from the previous pass (they include the covering frame)
  if (!keep && !(S.st & (S_NOCOV | S_PARTCARRY)) && S.X > ss + lo_c) {
    fent e;
    e.start = 0;
    e.ps = clamp_rel(S.cov_ps, ss);
    e.end = clamp_rel(S.X, ss);
    e.kw = S.cov_kw;
    L.fl[n++] = e;
  }
  const bool known = L.known != 0;
  const uint64_t lim = known ? L.Wn : NONE, hn = L.hn;
  bool past = L.past != 0, done = false, end = false;
  uint64_t cnt = 0, tail = 0;
  const uint32_t first_new = n;  // (the own frames of this pass come first, then any past the successor's entry)
  for (;;) {
    {
      // Fast path (many frames per segment): 32-bit segment-relative parse of
      // headers whose 14 bytes lie in LDS, in the batch and below the write
      // limit, before the successor's entry; anything else (a length of 2^31
      // or more, a limit, the segment end) goes to the general step below.
      uint64_t fstop = se - XYWS_MAX_FRAME_HEADER_SIZE + 1;
      const uint64_t hlim = P.hi < lim ? P.hi : lim;
      if (hlim < fstop + XYWS_MAX_FRAME_HEADER_SIZE - 1)
        fstop = hlim >= XYWS_MAX_FRAME_HEADER_SIZE - 1 ? hlim - (XYWS_MAX_FRAME_HEADER_SIZE - 1) : 0;
      if (known && !past && hn < fstop) fstop = hn;
      const uint64_t X0 = S.X;
      if (!(S.st & (S_PARTIAL | S_CUT)) && X0 >= ss && X0 < fstop) {
        const uint32_t st = (uint32_t)(fstop - ss);
        uint32_t x = (uint32_t)(X0 - ss), lx = 0, lps = 0, lkey = 0, lkw = 0, k = 0;
        while (x < st && n < G::FCAP) {
          uint32_t hl, plen, key, b01;
          if (!parse_rel<G>(L, x, hl, plen, key, b01)) break;  // >= 2^31: general step
          const uint32_t ps = x + hl;
          const uint32_t kw = rotr8(key, 0u - ps);  // aligned_key: ss is 16-byte aligned
          fent e;
          e.start = x; e.ps = ps; e.end = ps + plen; e.kw = kw;
          L.fl[n++] = e;
          lx = x; lps = ps; lkey = key; lkw = kw;
          x = ps + plen;
          k++;
        }
        if (k) {
          S.cov_start = ss + lx; S.cov_ps = ss + lps; S.X = ss + x;
          S.cov_key = lkey; S.cov_kw = lkw; S.st = 0;
          if (past) tail += k; else cnt += k;
        }
      }
    }
    const uint64_t X = S.X;
    if (known && !past && X >= hn) {  // the chain reached the successor's entry
      past = true;
      L.first_after = X;
      L.ok = X == hn;
    }
    if (X >= P.hi || (S.st & (S_PARTIAL | S_CUT))) { end = true; break; }
    if (X >= lim) { done = true; break; }
    if (X >= se || n >= G::FCAP) break;
    const hdr_info h = hdr_at(P, L, ss, X, lim);
    if (!h.hlen) {
      // incomplete: at the batch end (carry) or at the successor's write start
      const bool at_end = lim >= P.hi || X + XYWS_MAX_FRAME_HEADER_SIZE <= lim;
      S.st = (S.st & (S_NOCOV | S_CARRIED | S_HDRCARRY)) | (at_end ? S_PARTIAL : S_CUT);
      end = true;
      if (!at_end) { done = true; stat_add(P, ST_CUT, 1); }
      break;
    }
    const cstate F = frame_state(X, h);
    fent e;
    e.start = clamp_rel(X, ss);
    e.ps = clamp_rel(F.cov_ps, ss);
    e.end = clamp_rel(F.X, ss);
    e.kw = F.cov_kw;
    L.fl[n++] = e;
    if (past) tail++; else cnt++;
    S = F;
  }
  L.past = past;
  if (done) L.done = 1;
  if (end) L.end = 1;
  L.cnt += cnt;
  L.tail += tail;
  L.S = S;
  L.nfl = n;
  L.dense = n;
  if (P.fst) record_starts<G>(P, L, ss, first_new, (uint32_t)cnt);
  const bool seg_done = S.X >= se || end || done;
  L.pass_hi = seg_done ? G::SEG : (uint32_t)((S.X - ss) & ~15ull);
}

// Stride pass (wave 0, every lane; the first pass of a segment, before lane
// 0's serial chase). In a stream of equal frames the frame after X starts at
// X + F, F the size of the frame that ends at X; lane i parses the headers at
// X + (64j + i)*F, j < SP, from LDS (the serial chase's 32-bit parse, below
// the same stop). Position 0 is exact (X); position i is exact when
// positions 0..i-1 each hold a frame of exactly F bytes (induction from X),
// so ONE ballot accepts positions 0..m, m the first whose frame is not F
// bytes long (its start is exact too; its own size ends the step). A step
// decides up to 64*SP frames in one LDS round trip where the serial chase
// takes one hop per frame, and it
// is exact whatever the bytes: no accepted position is a guess. Steps repeat
// from the new X while one accepts STRIDE_MIN frames or more. Returns the
// list entries written (the covering frame first, as chase_pass writes it;
// 0: nothing accepted, the list untouched) and leaves L.S, L.cnt and the
// descriptor starts as chase_pass would: lane 0's serial chase continues
// from there (limits, the segment end, lengths of 2^31 or more).
constexpr uint32_t STRIDE_MIN = 8;
constexpr uint32_t SP = 4;  // stride-pass positions per lane (up to 256 frames per step)
template <class G>
XYWS_DEV uint32_t stride_pass(const run_params& P, lds_t<G>& L, uint64_t ss, uint32_t lane) {
  const cstate S0 = L.S;
  const uint64_t se = ss + G::SEG;
  const bool known = L.known != 0, past = L.past != 0;
  const bool dense_seg = L.dense >= 2 * G::NSB;
  if (past || S0.st != 0 || S0.X < ss || S0.X >= se || S0.X <= S0.cov_start) return 0;
  const uint64_t F = S0.X - S0.cov_start;
  if (F < 2 || F > G::SEG / STRIDE_MIN) return 0;
  // chase_pass's fast-path stop: headers wholly in LDS, in the batch, below
  // the write limit, before the successor's entry
  const uint64_t lim = known ? L.Wn : NONE;
  uint64_t fstop = se - XYWS_MAX_FRAME_HEADER_SIZE + 1;
  const uint64_t hlim = P.hi < lim ? P.hi : lim;
  if (hlim < fstop + XYWS_MAX_FRAME_HEADER_SIZE - 1)
    fstop = hlim >= XYWS_MAX_FRAME_HEADER_SIZE - 1 ? hlim - (XYWS_MAX_FRAME_HEADER_SIZE - 1) : 0;
  if (known && L.hn < fstop) fstop = L.hn;
  if (S0.X >= fstop) return 0;
  const uint64_t st = fstop - ss;
  // the covering frame's entry (chase_pass: when it reaches into the segment)
  const uint32_t n0 = S0.X > ss ? 1u : 0u;
  if (lane == 0 && n0) L.fl[0] = fent{0u, clamp_rel(S0.cov_ps, ss), clamp_rel(S0.X, ss), S0.cov_kw};
  uint32_t n = n0, total = 0, x = (uint32_t)(S0.X - ss), f = (uint32_t)F;
  bool uni = true;  // every accepted frame F bytes long (lattice_check)
  cstate S = S0;
  for (;;) {
    // SP positions per lane: frames x + (64*j + lane)*f, j < SP
    uint32_t pj[SP], hl[SP], pl[SP], ky[SP];
    uint64_t vm[SP], om[SP], mm[SP];
#pragma unroll
    for (uint32_t j = 0; j < SP; j++) {
      const uint64_t p64 = (uint64_t)x + (uint64_t)(64u * j + lane) * f;
      const bool v = p64 < st && n + 64u * j + lane < G::FCAP;
      pj[j] = (uint32_t)p64;
      hl[j] = pl[j] = ky[j] = 0;
      uint32_t b01 = 0;
      const bool ok = v && parse_rel<G>(L, pj[j], hl[j], pl[j], ky[j], b01);
      vm[j] = __ballot(v);
      om[j] = __ballot(ok);
      mm[j] = __ballot(ok && hl[j] + pl[j] == f);
    }
    // the first position without a match, in the order j = 0, 1, ...
    uint32_t m = 64u * SP, nv = 0;
    bool okm = false;
#pragma unroll
    for (int j = SP - 1; j >= 0; j--)
      if (mm[j] != ~0ull) {
        m = 64u * j + (uint32_t)__builtin_ctzll(~mm[j]);
        okm = ((om[j] >> (m & 63u)) & 1ull) != 0;
      }
#pragma unroll
    for (uint32_t j = 0; j < SP; j++) nv += (uint32_t)__builtin_popcountll(vm[j]);
    uint32_t a = okm ? m + 1 : m;  // (the first mismatch's start is exact: its own size ends the step)
    if (a > nv) a = nv;
    if (a == 0) break;
#pragma unroll
    for (uint32_t j = 0; j < SP; j++)
      if (64u * j + lane < a) {
        const uint32_t ps = pj[j] + hl[j];
        L.fl[n + 64u * j + lane] = fent{pj[j], ps, ps + pl[j], rotr8(ky[j], 0u - ps)};
      }
    // the last accepted frame is the chain state
    const uint32_t l = a - 1, ll = l & 63u, jl = l >> 6;
    uint32_t lp = 0, lhl = 0, lpl = 0, lkey = 0;
#pragma unroll
    for (uint32_t j = 0; j < SP; j++)
      if (jl == j) {
        lp = __builtin_amdgcn_readlane(pj[j], ll);
        lhl = __builtin_amdgcn_readlane(hl[j], ll);
        lpl = __builtin_amdgcn_readlane(pl[j], ll);
        lkey = __builtin_amdgcn_readlane(ky[j], ll);
      }
    S.cov_start = ss + lp;
    S.cov_ps = ss + lp + lhl;
    S.X = ss + lp + lhl + lpl;
    S.cov_key = lkey;
    S.cov_kw = rotr8(lkey, 0u - (lp + lhl));
    S.st = 0;
    n += a;
    total += a;
    x = lp + lhl + lpl;
    f = lhl + lpl;
    uni = uni && f == (uint32_t)F;
    if (a < STRIDE_MIN || x >= st || n >= G::FCAP) break;
  }
  if (lane == 0) {
    L.ar_f = uni ? (uint32_t)F : 0u;
    if (total) {
      L.S = S;
      L.cnt += total;
      if (P.fst) record_starts<G>(P, L, ss, n0, total);
    }
    // (a segment the dense pass would take and this pass did not cover: the
    // dense pass from the next segment on)
    if (dense_seg && total < 2 * G::NSB) L.sgood = 0;
  }
  return total ? n : 0u;
}

// Dense pass (many small frames): the segment's chase split over NSB
// sub-blocks of SB bytes (entries searched by 16 lanes each, chased by one
// lane each of wave 0), chased at once. Sub-block 0 starts
// from the exact state; sub-block b > 0 from its speculated entry, the
// earliest position in its first 512 bytes whose next 4 headers (32-bit parse
// in LDS) have client first bytes. Every chase starts exactly where the previous
// sub-block's chase leaves the previous sub-block, or the pass is abandoned
// (false, nothing of the chain state changed) and the serial chase runs: a
// chain is determined by its start, so sub-block b's frames are exact once its
// start is, by induction from sub-block 0. Entries go to per-sub-block sections
// of the frame list and are compacted (one per thread). A last header that
// does not fit the segment ends the pass (pass_hi) and the serial chase
// continues it; so does the serial chase from dstop, the successor's entry
// when it lies in the segment (no write limit lies below it).
template <class G>
XYWS_DEV bool dense_pass(const run_params& P, lds_t<G>& L, uint64_t ss, uint32_t tid_in, bool unm, bool past,
                         uint32_t dstop, bool rsv0 = false) {
  // (the lane index made opaque here: its LDS address math is recomputed per
  // pass instead of being hoisted out of the segment loop and spilled)
  uint32_t tid = tid_in;
  asm volatile("" : "+v"(tid));
  constexpr uint32_t NSB = G::NSB, SB = G::SB, SECT = G::SECT;
  constexpr uint32_t STOP = G::SEG - XYWS_MAX_FRAME_HEADER_SIZE + 1;  // headers wholly in LDS start below
  const uint32_t lane = tid & 63u, gl = lane & 15u, sb = (tid >> 6) * 4 + (lane >> 4);
  const cstate S0 = L.S;
  const uint32_t x0 = (uint32_t)(S0.X - ss);
  // sub-blocks starting below dstop (the successor's entry, or STOP) are chased
  const uint32_t nact = (dstop + SB - 1) / SB;
  const bool st_on = stats_on(P) && tid == 0;
  uint64_t tq = st_on ? __builtin_amdgcn_s_memtime() : 0;
  if (gl == 0) L.dent[sb] = sb == 0 ? x0 : NONE32;
  __syncthreads();
  if (st_on) tq = __builtin_amdgcn_s_memtime();
  // 1. speculated entries: each lane of the 16-lane group takes WIN/16 bytes
  //    and checks its candidates in order, one hop per loop iteration (a
  //    single loop: the wave steps every lane's current chain together)
  if (sb > 0 && sb < nact) {
    constexpr uint32_t WIN = SB < 512 ? SB : 512, PER = WIN / 16;
    static_assert(PER == 16 || PER == 32, "entry window: one or two 16-byte chunks per lane");
    const uint32_t a = sb * SB + gl * PER;
    uint32_t bits = chunk_candidates<G>(P, L, a, unm);
    if (PER == 32) bits |= chunk_candidates<G>(P, L, a + 16, unm) << 16;
    uint32_t p = NONE32, x = 0, h = 0;
    if (bits) { p = a + __builtin_ctz(bits); bits &= bits - 1; x = p; }
#pragma unroll 1
    while (p != NONE32) {
      // 4 client headers in a row, or 3 and a hop out of the segment (one
      // long hop proves little)
      const bool in = x < STOP;
      uint32_t hl = 0, plen = 0, key, b01;
      const bool ok = in && parse_rel<G>(L, x, hl, plen, key, b01) && cand_pair(b01 & 0xFFu, b01 >> 8, unm);
      if (in ? (ok && h == 3) : h >= 3) break;
      if (ok) {
        x += hl + plen;
        h++;
      } else if (bits) {
        p = a + __builtin_ctz(bits);
        bits &= bits - 1;
        x = p;
        h = 0;
      } else {
        p = NONE32;
      }
    }
    if (p != NONE32) atomicMin(&L.dent[sb], p);
  }
  __syncthreads();
  if (st_on) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    stat_add(P, ST_D_TENT, t - tq);
    tq = t;
  }
  // 2. one chase per sub-block, all in wave 0 (lane b: sub-block b; one wave
  //    stepping 64 chains issues a quarter of the instructions 16 waves
  //    stepping 4 chains each do)
  if (tid < NSB && tid >= nact) L.dcnt[tid] = 0;
  if (tid < nact) {
    const uint32_t sb = tid;
    uint32_t x = L.dent[sb], n = 0, lx = 0, lps = 0, lkey = 0, lkw = 0;
    bool fail = x == NONE32;
    const uint32_t end = (sb + 1) * SB;
    while (!fail && x < end && x < dstop) {
      uint32_t hl, plen, key, b01;
      if (n >= SECT || !parse_rel<G>(L, x, hl, plen, key, b01)) { fail = true; break; }
      const uint32_t ps = x + hl, kw = rotr8(key, 0u - ps);
      fent e;
      e.start = x; e.ps = ps; e.end = ps + plen; e.kw = kw;
      L.fl[sb * SECT + n] = e;
      n++;
      lx = x; lps = ps; lkey = key; lkw = kw;
      x = ps + plen;
    }
    // (a header starting at or past dstop ends the pass; only the last
    // chased sub-block can reach it)
    if (x < end && sb + 1 < nact) fail = true;
    L.dcnt[sb] = fail ? NONE32 : n;
    L.dexit[sb] = x;
    L.dlast[sb] = uint4{lx, lps, lkey, lkw};
  }
  __syncthreads();
  if (st_on) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    stat_add(P, ST_D_TCHASE, t - tq);
    tq = t;
  }
  // 3. validation and offsets (wave 0, one lane per sub-block)
  const bool cover = !(S0.st & (S_NOCOV | S_PARTCARRY)) && S0.X > ss;
  // list entries before the frames: the covering frame, or (rsv0) a slot
  // kept for one supplied later
  const uint32_t c0x = (cover || rsv0) ? 1u : 0u;
  if (tid < 64) {
    bool ok = true;
    uint32_t c = 0;
    if (lane < nact) {
      c = L.dcnt[lane];
      if (c == NONE32) {
        ok = false;
        if (stats_on(P)) stat_add(P, L.dent[lane] == NONE32 ? ST_D_NOENT : ST_D_CHASE, 1);
      } else if (lane > 0) {
        // the previous chase's exit must be one of this chase's frame starts
        // (usually the first; a false header just before a true one can land
        // on it): the frames from there on are exact
        const uint32_t xp = L.dexit[lane - 1];
        uint32_t j = 0;
        while (j < c && L.fl[lane * SECT + j].start < xp) j++;
        ok = j < c && L.fl[lane * SECT + j].start == xp;
        if (!ok && stats_on(P)) stat_add(P, ST_D_MISMATCH, 1);
        L.dent[lane] = j;  // entries skipped
        c -= j;
      } else {
        L.dent[0] = 0;
      }
      if (!ok) c = 0;
    }
    const bool all = __ballot(!ok) == 0;
    // exclusive prefix of the counts over the lanes
    uint32_t incl = c;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    const uint32_t total = __shfl(incl, 63) + c0x;
    if (lane < NSB) L.doff[lane] = c0x + incl - c;
    if (lane == 0) L.ccnt = all && total <= G::FCAP ? total : NONE32;
    if (lane == 0 && all && total > G::FCAP) stat_add(P, ST_D_OVF, 1);
    if (!all && lane == 0) {
      // a speculated entry was wrong (rare): walk the sub-blocks in order,
      // re-chasing each one whose frames do not contain the exact exit of the
      // previous one, from that exit; give up (serial chase) on overflow
      uint32_t tot = c0x;
      bool good = L.dcnt[0] != NONE32;
      if (good) { L.dent[0] = 0; L.doff[0] = tot; tot += L.dcnt[0]; }
      for (uint32_t b = 1; b < nact && good; b++) {
        const uint32_t xp = L.dexit[b - 1], cb = L.dcnt[b];
        uint32_t j = 0;
        if (cb != NONE32)
          while (j < cb && L.fl[b * SECT + j].start < xp) j++;
        if (cb == NONE32 || j >= cb || L.fl[b * SECT + j].start != xp) {
          uint32_t x = xp, n = 0, lx = 0, lps = 0, lkey = 0, lkw = 0;
          const uint32_t end = (b + 1) * SB;
          while (x < end && x < dstop) {
            uint32_t hl, plen, key, b01;
            if (n >= SECT || !parse_rel<G>(L, x, hl, plen, key, b01)) { good = false; break; }
            const uint32_t ps = x + hl, kw = rotr8(key, 0u - ps);
            fent e;
            e.start = x; e.ps = ps; e.end = ps + plen; e.kw = kw;
            L.fl[b * SECT + n] = e;
            n++;
            lx = x; lps = ps; lkey = key; lkw = kw;
            x = ps + plen;
          }
          if (x < end && b + 1 < nact) good = false;
          L.dcnt[b] = n;
          L.dexit[b] = x;
          if (n) L.dlast[b] = uint4{lx, lps, lkey, lkw};
          j = 0;
        }
        L.dent[b] = j;
        L.doff[b] = tot;
        tot += L.dcnt[b] - j;
      }
      L.ccnt = good && tot <= G::FCAP ? tot : NONE32;
    }
  }
  __syncthreads();
  if (st_on) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    stat_add(P, ST_D_TVAL, t - tq);
    tq = t;
  }
  const uint32_t total = L.ccnt;
  if (total == NONE32) return false;
  // 4. compaction (each thread moves at most one entry) and the chain state;
  //    descriptors requested: each thread also records its frame's start in
  //    the item's region (own frames only; the list is full: the re-walk)
  const uint32_t c0 = c0x, frames = total - c0;
  const bool rec_ok = P.fst && !past && L.nrec + frames <= P.rcap;
  {
    const uint32_t s = tid / SECT, j = tid % SECT, skip = L.dent[s];
    const bool mv = j >= skip && j < L.dcnt[s];
    const u32x4 e = mv ? *reinterpret_cast<const u32x4*>(&L.fl[tid]) : u32x4{0u, 0u, 0u, 0u};
    const uint64_t rbase = L.self * P.rcap + L.nrec;
    __syncthreads();
    if (mv) {
      const uint32_t pos = L.doff[s] + j - skip;
      *reinterpret_cast<u32x4*>(&L.fl[pos]) = e;
      if (rec_ok) P.fst[rbase + pos - c0] = ss + e.x;
    }
  }
  if (tid == 0) {
    if (cover) {
      fent e;
      e.start = 0;
      e.ps = clamp_rel(S0.cov_ps, ss);
      e.end = clamp_rel(S0.X, ss);
      e.kw = S0.cov_kw;
      L.fl[0] = e;
    } else if (rsv0) {
      L.fl[0] = fent{0u, 0u, 0u, 0u};
    }
    uint32_t last = nact - 1;  // the last sub-block with frames
    while (last > 0 && L.dcnt[last] == L.dent[last]) last--;
    const uint4 f = L.dlast[last];
    const uint32_t xe = L.dexit[nact - 1];
    if (frames) {
      cstate S;
      S.cov_start = ss + f.x; S.cov_ps = ss + f.y; S.X = ss + xe;
      S.cov_key = f.z; S.cov_kw = f.w; S.st = 0; S.pad = 0;
      L.S = S;
    }
    if (past) L.tail += frames; else L.cnt += frames;
    L.nfl = total;
    L.dense = total;
    if (rec_ok) L.nrec += frames;
    else if (P.fst && !past) flag_emit_slow(P);
    stat_add(P, ST_SEGS, 1);
    L.pass_hi = xe >= G::SEG ? G::SEG : (xe & ~15u);
  }
  __syncthreads();
  return true;
}

// Row table of one pass (wave 0, after lane 0's chase_pass; rows r = lane,
// lane + 64, ...): a row [r*1024, r*1024 + 1024) is FAST when every chunk in it
// is stored whole with the key word of one entry, SKIP when no chunk in it is
// stored, else the walk of its chunks starts at the last entry starting at or
// before the row (binary search).
constexpr uint32_t ROW_FAST = 1u << 16, ROW_SKIP = 1u << 17;
template <class G>
XYWS_DEV void build_rows(const fent* fl, uint2* rt, uint32_t nfl, uint32_t lo_c, uint32_t hi_c, uint32_t wl_r,
                         uint32_t wh_r, bool any, uint32_t lane) {
  for (uint32_t r = lane; r < G::SEG / 1024; r += 64) {
    const uint32_t R0 = r * 1024, R1 = R0 + 1024;
    uint32_t info = ROW_SKIP, kw = 0;
    if (any && nfl && R1 > lo_c && R0 < hi_c && R1 > wl_r && R0 < wh_r) {
      uint32_t x = 0, y = nfl;
      while (y - x > 1) {
        const uint32_t mid = (x + y) >> 1;
        if (fl[mid].start <= R0) x = mid; else y = mid;
      }
      const fent e = fl[x];
      const uint32_t ns = x + 1 < nfl ? fl[x + 1].start : 0xFFFFFFFFu;
      info = x;
      if (R0 >= lo_c && R1 <= hi_c && R0 >= wl_r && R1 <= wh_r && e.ps <= R0 && e.end >= R1 && ns >= R1) {
        info = e.kw ? ROW_FAST : ROW_SKIP;
        kw = e.kw;
      }
    }
    rt[r] = uint2{info, kw};
  }
}

// Chunks of the rows that are neither FAST nor SKIP (a frame boundary lies in
// the row), in a lane-private pass before the store loop (not unrolled: few
// registers live while the next segment's loads are in flight). Each of this
// lane's such chunks in [lo_c, hi_c) and wholly inside the write window [wl_r,
// wh_r) gets the words of every frame it overlaps XORed into its LDS copy
// (header bytes XOR 0: they stay as parsed) and bit k of the result: the store
// loop then stores it as it is, in the same instruction as its neighbours, so
// every line is written once (boundary chunks stored on their own after the
// loop wrote their lines a second time: c2 wrote 1.33x its batch). A chunk
// that crosses the window's edge gets bit k of `edge` (the byte path after
// the store loop). chunk_of(k, a, r, ok): the lane's k-th chunk offset, its
// 1 KiB row, and whether it exists.
template <class G, uint32_t NK, class ChunkOf>
XYWS_DEV uint32_t boundary_chunks(lds_t<G>& L, const fent* fl, const uint2* rt, uint32_t nfl, uint32_t lo_c,
                                  uint32_t hi_c, uint32_t wl_r, uint32_t wh_r, ChunkOf chunk_of, uint32_t& edge) {
  // the rows' classes first, all reads issued at once (one LDS round trip:
  // rows of whole-frame payload, the large-frame case, cost nothing more)
  uint32_t need = 0;
#pragma unroll
  for (uint32_t k = 0; k < NK; k++) {
    uint32_t a = 0, r = 0;
    bool ok = false;
    chunk_of(k, a, r, ok);
    const uint32_t info = __builtin_amdgcn_readfirstlane(rt[r].x);
    if (ok && !(info & (ROW_FAST | ROW_SKIP))) need |= 1u << k;
  }
  uint32_t put = 0;
  const uint32_t lane = __lane_id();
#pragma nounroll
  while (need) {
    const uint32_t k = __builtin_ctz(need);
    need &= need - 1;
    uint32_t a = 0, r = 0;
    bool ok = false;
    chunk_of(k, a, r, ok);
    // The row's frames at once (the wave holds one row: lane = chunk): lane j
    // reads entry g0 + j (g0 = the row's first entry, from the row table);
    // lane c's chunk starts in the last entry starting at or before it (g) and
    // meets every entry up to the last one starting before its end (gh): both
    // from the starts, broadcast one per step (no LDS round trip per entry).
    const uint32_t g0 = __builtin_amdgcn_readfirstlane(rt[r].x), R1 = r * 1024u + 1024u;
    const fent ej = g0 + lane < nfl ? fl[g0 + lane] : fent{0xFFFFFFFFu, 0u, 0u, 0u};
    const uint64_t inrow = __ballot(lane >= 1 && ej.start < R1);
    const bool mine = a >= lo_c && a < hi_c && a + 16 > wl_r && a < wh_r;
    const bool whole = a >= wl_r && a + 16 <= wh_r;
    if (mine && !whole) edge |= 1u << k;
    u32x4 m = {0u, 0u, 0u, 0u};
    if (inrow >> 63) {
      // (64 entries or more in the row: tiny frames) the walk from g0
      uint32_t g = g0;
      uint32_t ns = g + 1 < nfl ? fl[g + 1].start : 0xFFFFFFFFu;
      while (ns <= a) {
        g++;
        ns = g + 1 < nfl ? fl[g + 1].start : 0xFFFFFFFFu;
      }
      if (mine && whole) m = chunk_xor(fl, nfl, g, a);
    } else {
      uint32_t g = 0, gh = 0;
      for (uint64_t b = inrow; b; b &= b - 1) {
        const uint32_t j = (uint32_t)__builtin_ctzll(b);
        const uint32_t sj = __builtin_amdgcn_readlane(ej.start, j);
        if (sj <= a) g = j;
        if (sj < a + 16) gh = j;
      }
      const fent f0 = fl[g0 + g];
      const fent f1 = fl[g0 + g + (gh > g ? 1u : 0u)];
      m = span_key16(a, f0.ps, f0.end, f0.kw);
      if (gh > g) {
        m |= span_key16(a, f1.ps, f1.end, f1.kw);
        // (a third frame starting in the chunk: frames under 16 bytes)
        for (uint32_t h = g0 + g + 2; h <= g0 + gh; h++) {
          const fent f = fl[h];
          m |= span_key16(a, f.ps, f.end, f.kw);
        }
      }
      if (!(mine && whole)) m = u32x4{0u, 0u, 0u, 0u};
    }
    if (m.x | m.y | m.z | m.w) {
      u32x4* c = reinterpret_cast<u32x4*>(&L.seg[a]);
      *c = *c ^ m;
      put |= 1u << k;
    }
  }
  return put;
}

// Wait until run j's entry granule, claimed in this call, is published (lane
// 0); false when the bounded wait timed out (reported). The claimer is run j's
// own running workgroup, which computes its prologue without waiting for
// anything, so the wait ends; the bound only reports a bug.
XYWS_DEV bool wait_published(const run_params& P, uint32_t j, uint64_t E, uint64_t& a, uint64_t& b) {
  const uint64_t want = flag_published(E);
  uint32_t it = 0;
  for (;;) {
    granule_load(P.flags + 2 * (uint64_t)j, a, b);
    if (a == want || it >= SPIN) break;
    __builtin_amdgcn_s_sleep(2);
    it++;
  }
  if (it) stat_add(P, ST_SPIN, it);
  if (a != want) {
    atomicOr(P.head + 1, 2u);
    return false;
  }
  return true;
}

// The next run or piece after L.self that has an entry (lane 0), starting the
// search at flat index L.scan_j. Returns LK_FOUND with (hn, Wn, succ) (succ =
// nflat: none), or LK_GIVEUP with succ = the run whose entry is not published:
// its workgroup has not started (not every workgroup of the grid is resident,
// e.g. beside a concurrent decode, and waiting for one that is not could
// deadlock), or its bounded wait timed out (reported in the error word). A
// piece exists only when its run agreed to the split; its thief is running,
// so it is waited for. Never uses a granule not published in this call. A
// run given up on is bridged by finish_call.
enum { LK_FOUND = 0, LK_GIVEUP = 1 };
template <class G>
XYWS_DEV uint32_t lookup_successor(const run_params& P, lds_t<G>& L, uint64_t& hn, uint64_t& Wn, uint64_t& succ) {
  const uint64_t E = L.E, self = L.self;
  for (uint64_t j = L.scan_j; j < P.nflat; j++) {
    L.scan_j = j;
    uint64_t a, b;
    if (j & 1) {  // the piece of run j/2: only if that run agreed to the split
      const bool own = j == self + 1 && !(self & 1);
      if (own ? L.split_e == NONE : !split_is(st_load(P.split + 2 * (j >> 1)), E, SP_ACC)) continue;
      if (!wait_published(P, (uint32_t)j, E, a, b) || (b & (0x1FFFull << 51)) != granule_tag(E)) {
        succ = j;
        return LK_GIVEUP;
      }
    } else {
      granule_load(P.flags + 2 * j, a, b);
      // (test mode: odd runs give up on their successor at once)
      const bool test = (P.opts & XYWS_OPT_TEST_GIVEUP) && ((self >> 1) & 1u) && !(self & 1);
      if (test || (a >> 1) < E || (a != flag_published(E) && !wait_published(P, (uint32_t)j, E, a, b)) ||
          (b & (0x1FFFull << 51)) != granule_tag(E)) {
        if (a == flag_published(E) && (b & (0x1FFFull << 51)) != granule_tag(E)) atomicOr(P.head + 1, 8u);
        succ = j;
        return LK_GIVEUP;
      }
    }
    const uint64_t h = b & G_NONE;
    if (h != G_NONE) {
      hn = h;
      Wn = h + ((b >> 46) & 31u);
      succ = j;
      return LK_FOUND;
    }
  }
  hn = NONE;
  Wn = NONE;
  succ = P.nflat;
  return LK_FOUND;
}

// CH dropped stores (out-of-range offset: no memory traffic) after loads into
// `io`, so that on every path into the chain loop at least CH stores are
// younger than the loads: the compiler's wait before the fill is then
// vmcnt(CH), not vmcnt(0)
template <class G>
XYWS_DEV void dummy_stores(const run_params& P, uint64_t ss) {
  const __amdgpu_buffer_rsrc_t rz = seg_rsrc<G>(P, ss);
#pragma unroll
  for (uint32_t k = 0; k < G::CH; k++)
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, rz, OOB, k * G::NT * 16u, AUX_ST);  // distinct: not merged
}

// A run that will not split any more (lane 0; it is about to look up its
// successor, or it is done): close its split word, refusing a pending request.
XYWS_DEV void close_split(const run_params& P, uint64_t* sw, uint64_t E) {
  const unsigned long long fr = split_word(E, SP_FREE, 0);
  const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long*>(sw), fr,
                                           (unsigned long long)split_word(E, SP_CLS, 0));
  if (old != fr && split_is(old, E, SP_REQ)) st_store(sw, split_word(E, SP_CLS, 0));
}

// A steal request seen in the split word w the run loaded one segment earlier
// (lane 0, at the top of the segment at ss): the
// run keeps the current and the next segment and about half of the rest
// (less one segment, the thief's entry scan), the thief gets the tail.
template <class G>
XYWS_DEV void answer_split(const run_params& P, lds_t<G>& L, uint64_t ss, uint64_t w) {
  if (!split_is(w, L.E, SP_REQ)) return;
  uint64_t* sw = P.split + 2 * (L.self >> 1);
  const uint64_t rend = L.rng_end < P.hi ? L.rng_end : P.hi;
  const uint64_t i = (ss - L.rs) / G::SEG, nseg = (rend - L.rs + G::SEG - 1) / G::SEG;
  const uint64_t m = nseg > i ? nseg - i : 0;
  const uint64_t e = i + 2 + (m > 3 ? (m - 3) / 2 : 0);
  const uint64_t minp = (P.opts & XYWS_OPT_TEST_STEAL) ? 1 : XYWS_STEAL_MIN_PIECE;
  if (!L.known && e + minp <= nseg && e < (1u << 22)) {
    L.split_e = e;
    L.rng_end = L.rs + e * G::SEG;
    st_store(sw, split_word(L.E, SP_ACC, (uint32_t)e));
    stat_add(P, ST_STEAL_ACC, 1);
    stat_add(P, ST_STEAL_SEGS, nseg - e);
  } else {
    st_store(sw, split_word(L.E, SP_CLS, 0));
  }
  L.victim = 0;  // one answer per run
}

// Apply the chain in L.S (set by lane 0 together with L.known/hn/Wn/succ,
// L.rng_end and zeroed counters) from the segment at ss0: every byte in [wlo,
// write limit) is XORed with the key of the frame covering it, the write limit
// being the successor's W (looked up before the first segment at or past
// L.rng_end, unless known). The chase stops at the successor's W; L.ok tells
// whether it landed on its entry. A run (L.victim) answers steal requests on
// the way: its range end shrinks to the split.
// Lattice passes (run_chain; wave 0, after the chase of a single pass over the
// whole segment): when the list's entries 1, 2, ... start at X0, X0 + F, X0 +
// 2F, ... (equal frames, F >= 16: the stride pass's streams), the entry a
// chunk starts in is arithmetic, g = 1 + (a - X0) / F (0 before X0), and the
// chunk meets at most one more (g + 1): the store loop reads those two entries
// instead of the row table and the per-chunk walk (no row table is built).
// The stride pass's entries (below k0) are on the lattice when every frame it
// accepted was F bytes long (L.ar_f = F); the chase's few after them are
// checked here.
template <class G>
XYWS_DEV bool lattice_check(lds_t<G>& L, uint32_t nfl, uint32_t k0, uint32_t lane) {
  const uint32_t f = L.ar_f;
  if (nfl < 3 || f < 16 || f > G::SEG) return false;
  const uint32_t x0 = L.fl[1].start;
  if (L.fl[2].start - x0 != f) return false;
  bool ok = true;
  for (uint32_t i = (k0 > 1 ? k0 : 1u) + lane; i < nfl; i += 64) ok = ok && L.fl[i].start == x0 + (i - 1) * f;
  if (__ballot(!ok)) return false;
  if (lane == 0) L.ar_x0 = x0;
  return true;
}

// The two entries of chunk a on the lattice (x0, f; nfl entries): g, and
// whether entry g + 1 starts in the chunk.
XYWS_DEV uint32_t lattice_entry(uint32_t a, uint32_t x0, uint32_t f, float inv, uint32_t nfl, bool& two) {
  uint32_t g = 0;
  if (a >= x0) {
    const uint32_t d = a - x0;
    uint32_t i = (uint32_t)((float)d * inv);
    if ((i + 1) * f <= d) i++;
    else if (i * f > d) i--;
    g = 1 + i;
  }
  if (g > nfl - 1) g = nfl - 1;
  const uint32_t nxs = g == 0 ? x0 : x0 + g * f;  // entry g + 1's start
  two = g + 1 < nfl && nxs < a + 16;
  return g;
}

template <class G>
XYWS_DEV void run_chain(const run_params& P, lds_t<G>& L, seg_io<G>& io, uint32_t tid, uint64_t ss0,
                        bool in_lds, uint64_t wlo) {
  const bool stores = (P.opts & XYWS_OPT_PARSE_ONLY) == 0;
  const uint64_t wl = wlo > P.lo ? wlo : P.lo;
  // Pipeline: the registers of `io` always hold the loads of the segment the
  // next iteration fills into LDS, issued one iteration ahead; every pass
  // issues exactly CH stores per lane (skipped chunks go to an out-of-range
  // offset), so each fill waits for its loads only (vmcnt counts loads and
  // stores together, in issue order) while the previous segment's stores drain.
  if (!in_lds && io.pf != ss0) io.issue(P, ss0, tid, L.known ? L.Wn : NONE);
  dummy_stores<G>(P, ss0);
  // stats builds: wave 0 accumulates phase cycles in registers, flushed once
  const bool st_on = stats_on(P) && tid < 64;
  uint64_t tm = st_on ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t acc_tail = 0, acc_fill = 0, acc_pf = 0, acc_cp = 0, acc_sync = 0, acc_xor = 0;
#define XYWS_STAMP(acc)                                 \
  do {                                                  \
    if (st_on) {                                        \
      const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
      acc += t_ - tm;                                   \
      tm = t_;                                          \
    }                                                   \
  } while (0)
  // Once the next segment lies past the run's range the write limit is the
  // successor's W (its prologue published it long ago): looked up before the
  // next segment's prefetch is decided. No split is agreed after that.
  auto lookup = [&](uint64_t nxt) {
    if (tid == 0 && !L.known && nxt >= L.rng_end) {
      const uint64_t t0 = stats_on(P) ? __builtin_amdgcn_s_memtime() : 0;
      if (L.victim) {
        close_split(P, P.split + 2 * (L.self >> 1), L.E);
        L.victim = 0;
      }
      uint64_t hn = NONE, Wn = NONE, succ = P.nflat;
      if (lookup_successor(P, L, hn, Wn, succ) == LK_GIVEUP) {
        // unknown successor: write up to the own range end only and leave
        // the rest to finish_call (never a stale record)
        L.hn = NONE; L.Wn = L.rng_end; L.succ = succ; L.known = 1; L.tmo = 1;
      } else {
        L.hn = hn; L.Wn = Wn; L.succ = succ; L.known = 1;
      }
      if (stats_on(P)) stat_add(P, ST_T_WAIT, __builtin_amdgcn_s_memtime() - t0);
    }
  };
  lookup(ss0 + G::SEG);
  uint64_t split_w = L.split_poll[0];  // the run's split word as last read (lane 0)
  for (uint64_t ss = ss0;; ss += G::SEG) {
    const uint64_t nx = ss + G::SEG;
    __syncthreads();  // the previous segment's LDS reads are done; L control words visible
    XYWS_STAMP(acc_tail);
    const bool filled = !(in_lds && ss == ss0);
    if (filled) {
#pragma unroll
      for (uint32_t k = 0; k < G::CH; k++)
        *reinterpret_cast<u32x4*>(&L.seg[(k * G::NT + tid) * 16u]) = io.e[k];
      io.pf = NONE;
      // (the prefetch registers are free here: the lane-0 work of a run that
      // can be split goes where they are dead)
      asm volatile("" ::: "memory");
      if (tid == 0 && L.victim) answer_split<G>(P, L, ss, split_w);
    }
    __syncthreads();
    XYWS_STAMP(acc_fill);
    const bool known = L.known != 0;
    const uint64_t wlim = known ? L.Wn : L.rng_end;
    const uint64_t whi = wlim < P.hi ? wlim : P.hi;
    const bool fin0 = (L.end || L.done) && nx >= whi;
    const bool pf = nx < P.hi && nx < wlim && !fin0 && io.pf != nx;
    if (tid == 0 && L.victim && filled) {
      // progress for thieves, and the split word for the next iteration
      // (both before the prefetch)
      const uint32_t r = (uint32_t)(L.self >> 1);
      st_store(P.prog + r, (L.E << 24) | ((ss - L.rs) / G::SEG));
      // (a plain load into a register: the compiler waits for it where it is
      // used, next iteration, by counting; an LDS-DMA here made it wait
      // vmcnt(0), i.e. for the whole prefetch, at the next barrier)
      split_w = st_load(P.split + 2 * r);
    }
    // (issuing each chunk's next load right after its LDS write made hipcc wait
    // for the new loads inside the fill: the prefetch goes after the barrier)
    if (pf) io.issue(P, nx, tid, known ? wlim : NONE);
    XYWS_STAMP(acc_pf);
    const __amdgpu_buffer_rsrc_t rs = seg_rsrc<G>(P, ss);
    uint32_t lo_c = 0, keep = 0;
    for (;;) {
      // write window [wl, whi) relative to the segment (32-bit compares below)
      const uint32_t wl_r = wl > ss ? (wl - ss < G::SEG ? (uint32_t)(wl - ss) : G::SEG) : 0u;
      const uint32_t wh_r = whi > ss ? (whi - ss < G::SEG ? (uint32_t)(whi - ss) : G::SEG) : 0u;
      const bool any = stores && !(P.opts & XYWS_OPT_NO_STORE) && wl_r < wh_r;
      // the dense pass where the previous pass found many frames and no limit
      // lies in this segment (the serial chase below otherwise, or after it)
      bool dense = false;
      if (lo_c == 0 && keep == 0 && L.dense >= 2 * G::NSB && !L.sgood) {
        const cstate S0 = L.S;
        const bool kn = L.known != 0, pst = L.past != 0;
        const uint64_t se14 = ss + G::SEG + XYWS_MAX_FRAME_HEADER_SIZE;
        constexpr uint32_t STOP = G::SEG - XYWS_MAX_FRAME_HEADER_SIZE + 1;
        // the successor's entry in this segment: the pass stops there (the
        // serial chase below crosses it), beyond its first two sub-blocks
        const bool hin = kn && !pst && L.hn < se14;
        const uint32_t dstop = hin ? (L.hn - ss < STOP ? (uint32_t)(L.hn - ss) : STOP) : STOP;
        if (!(S0.st & (S_PARTIAL | S_CUT)) && S0.X >= ss && S0.X < ss + G::SB && P.hi >= se14 &&
            (!kn || (hin ? (L.hn >= ss + 2 * G::SB && L.Wn >= L.hn) : L.Wn >= se14)))
          dense = dense_pass<G>(P, L, ss, tid, (P.opts & XYWS_OPT_UNMASKED_HINT) != 0, pst, dstop);
      }
      if (tid < 64) {
        // lane 0 chases; then wave 0 classifies the rows (the other waves wait
        // at the barrier with their prefetch in flight: work here is hidden,
        // work in the store loop below is not)
        const uint64_t t_r0 = st_on ? __builtin_amdgcn_s_memtime() : 0;
        // the stride pass first (exact; regular frames), then lane 0's chase
        uint32_t k0 = keep;
        if (!dense && lo_c == 0 && keep == 0) {
          k0 = stride_pass<G>(P, L, ss, tid);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          if (st_on && tid == 0) stat_add(P, ST_T_STRIDE, __builtin_amdgcn_s_memtime() - t_r0);
        }
        if (tid == 0 && !dense) chase_pass(P, L, ss, lo_c, k0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t t_r1 = st_on ? __builtin_amdgcn_s_memtime() : 0;
        // (only after a stride pass: mixed sizes skip the check)
        const bool lat = k0 != 0 && lo_c == 0 && L.pass_hi >= G::SEG && !(P.opts & XYWS_OPT_NO_LATTICE) &&
                         lattice_check<G>(L, L.nfl, k0, tid);
        if (tid == 0) L.ar = lat;
        if (!lat) build_rows<G>(L.fl, L.rt, L.nfl, lo_c, L.pass_hi, wl_r, wh_r, any, tid);
        if (st_on && tid == 0) {
          stat_add(P, ST_T_SER, t_r1 - t_r0);
          stat_add(P, ST_T_ROWS, __builtin_amdgcn_s_memtime() - t_r1);
        }
      }
      XYWS_STAMP(acc_cp);
      // Large frames (serial chase): the next segment's loads and this run's
      // earlier stores drain before this segment's stores go out (measured
      // ~0.6 % faster on c3 than letting them overlap); the dense pass never
      // waits here (its chase is what the prefetch hides).
      if (!dense && !(P.opts & XYWS_OPT_RUNS_NOWAIT)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      XYWS_STAMP(acc_sync);
      const uint32_t nfl = L.nfl, hi_c = L.pass_hi;
      // Per chunk: a FAST row XORs with one scalar key word, a SKIP row stores
      // nothing; otherwise the lane walks the sorted, contiguous frame list from
      // the row's entry: entry g covers the chunk when no later entry starts in
      // it and its payload spans it (one key word for all four dwords). Every
      // chunk issues exactly one store here (dropped ones to the out-of-range
      // offset); chunks holding a header or a frame boundary, and the batch's
      // first/last chunk, are left to the loop after it (few registers live in
      // this unrolled loop: the next segment's loads are in flight).
      uint32_t edge = 0;
      const uint32_t wave = tid >> 6;
      if (L.ar) {
        // a lattice pass: each chunk's two entries by arithmetic (lattice_entry)
        const uint32_t x0 = L.ar_x0, f = L.ar_f;
        const float inv = 1.0f / (float)f;
        u32x4 dprev = {0u, 0u, 0u, 0u};
#pragma unroll 2
        for (uint32_t k = 0; k < G::CH; k++) {
          const uint32_t a = (k * G::NT + tid) * 16u;
          bool two = false;
          const uint32_t g = lattice_entry(a, x0, f, inv, nfl, two);
          const fent f0 = L.fl[g];
          const fent f1 = L.fl[two ? g + 1 : g];
          const u32x4 v = *reinterpret_cast<const u32x4*>(&L.seg[a]);
          u32x4 m;
          m = span_key16(a, f0.ps, f0.end, f0.kw);
          if (two) {
            m |= span_key16(a, f1.ps, f1.end, f1.kw);
          }
          const bool whole = a >= wl_r && a + 16 <= wh_r;
          if (!whole && a + 16 > wl_r && a < wh_r) edge |= 1u << k;
          const uint32_t off = whole && (m.x | m.y | m.z | m.w) ? tid * 16u : OOB;
          const u32x4 d = v ^ m;
          __builtin_amdgcn_raw_buffer_store_b128(d, rs, off, k * G::NT * 16u, AUX_ST);
          asm volatile("" ::"v"(dprev.x), "v"(dprev.y), "v"(dprev.z), "v"(dprev.w));
          dprev = d;
        }
        asm volatile("s_nop 1" ::"v"(dprev.x), "v"(dprev.y), "v"(dprev.z), "v"(dprev.w));
      } else {
      const uint32_t put = boundary_chunks<G, G::CH>(
          L, L.fl, L.rt, nfl, lo_c, hi_c, wl_r, wh_r,
          [&](uint32_t k, uint32_t& a, uint32_t& r, bool& ok) {
            a = (k * G::NT + tid) * 16u;
            r = k * (G::NT / 64) + wave;
            ok = true;
          },
          edge);
      u32x4 dprev = {0u, 0u, 0u, 0u};
      // software pipeline: chunk k+1's row word and bytes are read from LDS
      // before chunk k's store
      uint2 rw_n = L.rt[wave];
      u32x4 v_n = *reinterpret_cast<const u32x4*>(&L.seg[tid * 16u]);
#pragma unroll
      for (uint32_t k = 0; k < G::CH; k++) {
        const uint32_t a = (k * G::NT + tid) * 16u;
        const uint2 rw = rw_n;
        const u32x4 v = v_n;
        if (k + 1 < G::CH) {
          rw_n = L.rt[(k + 1) * (G::NT / 64) + wave];
          v_n = *reinterpret_cast<const u32x4*>(&L.seg[((k + 1) * G::NT + tid) * 16u]);
        }
        const uint32_t info = __builtin_amdgcn_readfirstlane(rw.x);
        const uint32_t kw = __builtin_amdgcn_readfirstlane(rw.y);
        u32x4 m;
        uint32_t off;
        if (info & ROW_FAST) {
          m = u32x4{kw, kw, kw, kw};
          off = tid * 16u;
        } else if (info & ROW_SKIP) {
          m = u32x4{0u, 0u, 0u, 0u};
          off = OOB;
        } else {
          // (XORed in LDS already when bit k of put is set: boundary_chunks)
          m = u32x4{0u, 0u, 0u, 0u};
          off = ((put >> k) & 1u) ? tid * 16u : OOB;
          (void)a;
        }
        const u32x4 d = v ^ m;
        __builtin_amdgcn_raw_buffer_store_b128(d, rs, off, k * G::NT * 16u, AUX_ST);
        // hipcc (ROCm 7.2, gfx950) may overwrite a dwordx4 store's data VGPRs
        // in the very next instruction; later lanes then store the new value
        // (seen as wrong bytes in dword 0, lanes 12-15 of each 16). The data
        // stays live until after the next chunk's store (an empty asm use, no
        // memory clobber: the next chunk's LDS reads may still be hoisted).
        asm volatile("" ::"v"(dprev.x), "v"(dprev.y), "v"(dprev.z), "v"(dprev.w));
        dprev = d;
      }
      asm volatile("s_nop 1" ::"v"(dprev.x), "v"(dprev.y), "v"(dprev.z), "v"(dprev.w));
      }
#pragma nounroll
      while (edge) {  // chunks with a frame boundary, and the batch's first/last chunk
        const uint32_t k = __builtin_ctz(edge);
        edge &= edge - 1;
        const uint32_t a = (k * G::NT + tid) * 16u;
        uint32_t x = 0, y = nfl;
        while (y - x > 1) {
          const uint32_t mid = (x + y) >> 1;
          if (L.fl[mid].start <= a) x = mid; else y = mid;
        }
        const u32x4 m = chunk_xor(L.fl, nfl, x, a);
        if ((m.x | m.y | m.z | m.w) == 0u) continue;
        if (a >= wl_r && a + 16 <= wh_r) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(&L.seg[a]);
          __builtin_amdgcn_raw_buffer_store_b128(v ^ m, rs, tid * 16u, k * G::NT * 16u, AUX_ST);
          asm volatile("s_nop 1" ::: "memory");
          continue;
        }
        const uint64_t A = ss + a;
#pragma nounroll
        for (uint32_t t = 0; t < 16; t++) {  // only the bytes in [wl, whi)
          const uint64_t q = A + t;
          const uint32_t mw = t < 4 ? m.x : t < 8 ? m.y : t < 12 ? m.z : m.w;
          const uint8_t kb = (uint8_t)(mw >> (8u * (t & 3u)));
          if (kb && q >= wl && q < whi) P.base[q] = L.seg[a + t] ^ kb;
        }
      }
      XYWS_STAMP(acc_xor);
      if (hi_c >= G::SEG) break;
      __syncthreads();  // the list is rebuilt for the next pass
      if (tid == 0) {   // entries reaching past hi_c (tiny frames can share its chunk) carry over
        uint32_t c = nfl;
        while (c > 0 && L.fl[c - 1].end > hi_c) c--;
        for (uint32_t i = c; i < nfl; i++) L.fl[i - c] = L.fl[i];
        L.keepn = nfl - c;
      }
      __syncthreads();
      keep = L.keepn;
      lo_c = hi_c;
    }
    // continue while bytes below the write limit remain
    const bool fin = (L.end || L.done) && nx >= whi;
    if (nx >= P.hi || nx >= wlim || fin) break;
    lookup(nx + G::SEG);
  }
  if (st_on && tid == 0) {
    stat_add(P, ST_T_TAIL, acc_tail);
    stat_add(P, ST_T_FILL, acc_fill);
    stat_add(P, ST_T_PF, acc_pf);
    stat_add(P, ST_T_CP, acc_cp);
    stat_add(P, ST_T_CHASE, acc_sync);
    stat_add(P, ST_T_XOR, acc_xor);
  }
#undef XYWS_STAMP
  __syncthreads();
}

// ---------------------------------------------------------------- prologue
// Earliest position of run `run`'s range whose chain of KHDR headers is
// plausible (lane 0 returns it through L.aux0; NONE if there is none). Leaves
// the segment it was found in (L.aux1) in LDS.
//
// A candidate's chain from header position x with i headers verified (need:
// the headers its length form asks for, set at the first): 0 implausible, 1
// plausible, 2 undecided (only when !mem: its next header is not readable
// from the LDS copy of [ss, ss + SEGX)); x, i and need are left where it
// stopped.
template <class G>
XYWS_DEV uint32_t chain_follow(const run_params& P, const lds_t<G>& L, uint64_t ss, uint64_t& x, uint32_t& i,
                               uint32_t& need, bool unm, bool mem) {
  for (; i < need; i++) {
    // a chain that ends with the batch counts after two verified headers (one
    // header whose length jumps past the batch end proves nothing: random
    // bytes 0xFF 0x00 0x00 ... pass as a 64-bit length below 2^46 often enough)
    if (x >= P.hi) return i >= 2;
    if (!mem && (x < ss || x - ss + XYWS_MAX_FRAME_HEADER_SIZE > G::SEGX)) return 2u;
    const hdr_info h = hdr_at(P, L, ss, x, NONE);
    if (!h.hlen) return i >= 2;   // a header cut by the batch end
    if (!plausible(h, unm)) return 0u;
    if (i == 0) {
      const uint32_t ext = h.hlen - 2 - ((h.status & XYWS_ST_UNMASKED) ? 0u : 4u);
      need = ext == 8 ? KHDR_127 : ext == 2 ? KHDR_126 : KHDR_7;
    }
    x = sat_add(x + h.hlen, h.plen);
  }
  return 1u;
}
template <class G>
XYWS_DEV uint32_t chain_plausible(const run_params& P, const lds_t<G>& L, uint64_t ss, uint64_t q, bool unm,
                                  bool mem) {
  uint64_t x = q;
  uint32_t i = 0, need = KHDR_7;
  return chain_follow<G>(P, L, ss, x, i, need, unm, mem);
}

// Second-level filter for the candidate at segment offset p (cheap, from LDS):
// false only when the header after it (7-bit or 126 form) lies in the segment
// and the batch and fails cand_pair, i.e. when its chain is certainly
// implausible (cand_pair is implied by plausible()).
template <class G>
XYWS_DEV bool second_hop_ok(const run_params& P, const lds_t<G>& L, uint64_t ss, uint32_t p, bool unm) {
  const uint32_t b1 = L.seg[p + 1], l7 = b1 & 0x7Fu;
  uint32_t nxt;
  if (l7 < 126) nxt = p + 2 + (unm ? 0u : 4u) + l7;
  else if (l7 == 126) nxt = p + 4 + (unm ? 0u : 4u) + (((uint32_t)L.seg[p + 2] << 8) | L.seg[p + 3]);
  else return true;
  if (nxt + 2 > G::SEGX || ss + nxt + 2 > P.hi) return true;
  return cand_pair(L.seg[nxt], L.seg[nxt + 1], unm);
}

// Prologue scan of the segment at ss, in LDS (see find_entry): L.best = the
// earliest offset whose chain of KHDR headers is plausible (0xFFFFFFFF: none).
//  first for the segment's first NT chunks, then (no winner) for the rest
//  (w0: both in one pass, after calls of large frames of mixed sizes):
//  1. every lane filters its chunks: candidate bits (SWAR) and the cheap
//     second-hop test; survivors go to an LDS list;
//  2. survivors' chains, one per lane, followed in LDS; chains leaving the
//     segment are listed as undecided;
//  then 3. undecided survivors below the best so far: chains followed through
//     memory (one memory latency per segment).
// A list overflow (e.g. a stream of 2-byte frames) falls back to each lane
// checking its own candidates in order through memory.
template <class G>
XYWS_DEV void scan_segment(const run_params& P, lds_t<G>& L, uint64_t ss, uint32_t tid, bool unm, bool w0) {
  const bool st_on = stats_on(P) && tid == 0;
  uint64_t tq = st_on ? __builtin_amdgcn_s_memtime() : 0, a_filt = 0, a_chk = 0, nwin = 0, nsurv = 0;
  if (tid == 0) { L.ucnt = 0; L.ovf = 0; }
  // candidate offsets below qlim: the header fits the segment, the byte is in the batch
  const uint64_t rel_hi = P.hi - ss;
  const uint32_t qlim = rel_hi < G::SEG - XYWS_MAX_FRAME_HEADER_SIZE + 1 ? (uint32_t)rel_hi
                                                                          : G::SEG - XYWS_MAX_FRAME_HEADER_SIZE + 1;
  // Candidate bits of chunk k (segment offset (k*NT + tid)*16: conflict-free
  // LDS reads), bit 8*b + h + i = byte b of dword i (h: a 4-bit lane of the
  // packed word).
  // (32-bit bounds only: a 64-bit per-lane position here was a spilled
  // value whose reload waited for the next segment's loads in flight)
  const uint32_t rhi = rel_hi < 0xFFFFFFFFull ? (uint32_t)rel_hi : 0xFFFFFFFFu;
  auto chunk_bits = [&](uint32_t k, uint32_t h) -> uint32_t {
    const uint32_t a = (k * G::NT + tid) * 16u;
    if (a >= rhi) return 0u;
    const u32x4 v = *reinterpret_cast<const u32x4*>(L.seg + a);
    const uint32_t w4 = *reinterpret_cast<const uint32_t*>(L.seg + a + 16);
    uint32_t c = (cand_bytes(v.x, v.y, unm) >> (7 - h)) | (cand_bytes(v.y, v.z, unm) >> (6 - h)) |
                 (cand_bytes(v.z, v.w, unm) >> (5 - h)) | (cand_bytes(v.w, w4, unm) >> (4 - h));
    if (a + 16 > qlim) {
      uint32_t keep = 0;
#pragma unroll 1
      for (uint32_t t = 0; a + t < qlim && t < 16; t++) keep |= 1u << (8u * (t & 3u) + h + (t >> 2));
      c &= keep;
    }
    return c;
  };
  auto survivor = [&](uint32_t pos) {
    if (second_hop_ok<G>(P, L, ss, pos, unm)) {
      const uint32_t slot = atomicAdd(&L.ccnt, 1u);
      if (slot < G::SCAP) L.sl[slot] = pos;
    }
  };
  // survivors' chains in LDS, one per lane; chains leaving the segment are
  // listed as undecided; true when the scan is over (a winner, or overflow)
  auto check = [&]() -> bool {
    __syncthreads();
    const uint32_t n = L.ccnt;
    if (st_on) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      a_filt += t - tq; tq = t; nwin++; nsurv += n;
    }
    if (n > G::SCAP) {
      if (tid == 0) L.ovf = 1;
    } else {
      // (i is opaque to the compiler: a hoisted, spilled &L.sl[tid] would be
      // reloaded behind a vmcnt(0) that waits for the prefetch in flight)
      uint32_t i0 = tid;
      asm volatile("" : "+v"(i0));
      for (uint32_t i = i0; i < n; i += G::NT) {
        const uint32_t pos = L.sl[i];
        if (pos > __hip_atomic_load(&L.best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) continue;
        const uint32_t r = chain_plausible(P, L, ss, ss + pos, unm, false);
        if (r == 1u) {
          atomicMin(&L.best, pos);
        } else if (r == 2u) {
          const uint32_t u = atomicAdd(&L.ucnt, 1u);
          if (u < G::UCAP) L.ul[u] = pos;
          else L.ovf = 1;
        }
      }
    }
    __syncthreads();
    if (st_on) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      a_chk += t - tq; tq = t;
    }
    return L.ovf || L.best != 0xFFFFFFFFu;
  };
  // Window 0 (the first NT chunks, 16 KiB for 1024 lanes) alone first: a
  // chain usually starts within one frame of the range start. Then the rest
  // of the segment in one pass, each lane's candidates in one loop (a wave
  // iterates as often as its busiest lane). (!w0: one pass for the whole
  // segment: large frames leave window 0 empty, its check is one more round
  // of barriers and LDS chains per segment.)
  if (tid == 0) L.ccnt = 0;
  __syncthreads();
  {
    uint32_t c = chunk_bits(0, 0);
    while (c) {
      const uint32_t t = __builtin_ctz(c);
      c &= c - 1;
      survivor(tid * 16u + 4u * (t & 3u) + (t >> 3));
    }
  }
  if (st_on) stat_add(P, ST_X_W0, __builtin_amdgcn_s_memtime() - tq);
  const bool over = w0 ? check() : false;
  bool rest = false;
  if constexpr (G::CH > 1) rest = !over && ss + G::NT * 16u < P.hi;
  if constexpr (G::CH > 1) if (rest) {
    if (w0) {
      if (tid == 0) L.ccnt = 0;
      __syncthreads();
    }
    // chunks 1..CH-1 packed two per word: m[j] holds chunks 2j+1 (h = 0) and 2j+2 (h = 4)
    constexpr uint32_t NM = G::CH / 2;
    uint32_t m[NM > 0 ? NM : 1];
#pragma unroll
    for (uint32_t j = 0; j < NM; j++)
      m[j] = chunk_bits(2 * j + 1, 0) | (2 * j + 2 < G::CH ? chunk_bits(2 * j + 2, 4) : 0u);
    uint64_t tb = 0;
    if (st_on) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      tb = __builtin_amdgcn_s_memtime();
      stat_add(P, ST_X_BITS, tb - tq);
    }
    uint32_t any = 0;
#pragma unroll
    for (uint32_t j = 0; j < NM; j++) any |= m[j];
    while (any) {
      uint32_t b = m[0], g = 0;
#pragma unroll
      for (uint32_t j = NM - 1; j >= 1; j--) {
        if (m[j]) { b = m[j]; g = j; }  // the lowest non-empty word wins
      }
      if (m[0]) { b = m[0]; g = 0; }
      const uint32_t t = __builtin_ctz(b);
      const uint32_t bit = b & (0u - b);
#pragma unroll
      for (uint32_t j = 0; j < NM; j++)
        if (g == j) m[j] &= ~bit;
      any = 0;
#pragma unroll
      for (uint32_t j = 0; j < NM; j++) any |= m[j];
      const uint32_t k = 2 * g + 1 + ((t >> 2) & 1u);
      survivor((k * G::NT + tid) * 16u + 4u * (t & 3u) + (t >> 3));
    }
    if (st_on) stat_add(P, ST_X_SURV, __builtin_amdgcn_s_memtime() - tb);
    (void)check();
  }
  if (!rest && !w0) (void)check();  // (window 0 was the whole pass: its own check)
  if (st_on) {
    stat_add(P, ST_P_TCOMP, a_filt); stat_add(P, ST_P_TCHECK, a_chk);
    stat_add(P, ST_P_WIN, nwin); stat_add(P, ST_P_CAND, nsurv); stat_add(P, ST_P_UND, L.ucnt);
  }
  if (L.ovf) {
    // a list overflowed (e.g. a stream of 2-byte frames): each lane checks its
    // own candidates in order, through memory, from scratch
    __syncthreads();
    if (tid == 0) L.best = 0xFFFFFFFFu;
    __syncthreads();
#pragma unroll 1
    for (uint32_t k = 0; k < G::CH; k++) {
      const uint32_t a = (k * G::NT + tid) * 16u;
      uint32_t b = ss + a < P.hi ? chunk_candidates<G>(P, L, a, unm) : 0u;
      bool hit = false;
      while (b) {
        const uint32_t t = __builtin_ctz(b);
        b &= b - 1;
        const uint32_t pos = a + t;
        if (pos > __hip_atomic_load(&L.best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) { hit = true; break; }
        if (chain_plausible(P, L, ss, ss + pos, unm, true) == 1u) {
          atomicMin(&L.best, pos);
          hit = true;
          break;
        }
      }
      if (hit) break;
    }
    __syncthreads();
    return;
  }
  // 3. undecided candidates below the best: chains through memory, all at once
  const uint32_t nu = L.ucnt, best = L.best;
  if (nu) {
    for (uint32_t i = tid; i < nu; i += G::NT) {
      const uint32_t pos = L.ul[i];
      if (pos < best && chain_plausible(P, L, ss, ss + pos, unm, true) == 1u) atomicMin(&L.best, pos);
    }
    __syncthreads();
    if (st_on) stat_add(P, ST_P_TRES, __builtin_amdgcn_s_memtime() - tq);
  }
}

template <class G>
XYWS_DEV void find_entry(const run_params& P, lds_t<G>& L, seg_io<G>& io, uint32_t tid, uint64_t rb,
                         uint64_t re) {
  const bool unm = (P.opts & XYWS_OPT_UNMASKED_HINT) != 0;
  // (after a call of large frames of mixed sizes: no window-0 pass)
  const bool big = P.bigscan != 0;
  if (re > P.hi) re = P.hi;
  if (tid == 0) L.aux0 = NONE;
  uint64_t tp = (stats_on(P) && tid == 0) ? __builtin_amdgcn_s_memtime() : 0;
  for (uint64_t ss = rb; ss < re; ss += G::SEG) {
    __syncthreads();
    io.fill(P, L, ss, tid);
    if (tid == 0) { L.best = 0xFFFFFFFFu; L.aux1 = ss; }
    __syncthreads();
    if (stats_on(P) && tid == 0) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      stat_add(P, ST_P_FILL, t - tp);
      tp = t;
    }
    // the next segment's loads fly during the scan: the chain starts there when
    // the entry is in this segment, the scan continues there when it is not
    // (HBM would idle during the scan otherwise; the few header reads from
    // memory below and the publish's vmcnt(0) wait for them)
    if (ss + G::SEG < P.hi && !(P.opts & XYWS_OPT_DIAG)) io.issue(P, ss + G::SEG, tid);
    // Lattice entry: when the previous call's frames were all F bytes long
    // (P.pfs), the first frame start at or after rb on the lattice X0 + kF (X0:
    // the batch's first frame start, after the carried frame) is tried first:
    // it wins when its header opens a frame of exactly F bytes and its chain
    // is plausible (the scan's own test). A speculation like the scan's
    // winner: the predecessor's exact chain checks it at the hand-over.
    if (P.pfs && ss == rb) {
      if (tid == 0) {
        const xyws_carry* cz = P.cin_user ? P.cin_user : &k_zero_carry;
        uint64_t c0;
        const cstate S0 = initial_state(P, cz, c0);
        const uint64_t F = P.pfs, x0 = S0.X;
        if (!(S0.st & (S_PARTIAL | S_PARTCARRY)) && x0 < P.hi) {
          const uint64_t q = rb <= x0 ? x0 : x0 + (rb - x0 + F - 1) / F * F;
          if (q >= ss && q + XYWS_MAX_FRAME_HEADER_SIZE <= ss + G::SEG && q < re) {
            const hdr_info h = hdr_at(P, L, ss, q, NONE);
            if (h.hlen && (uint64_t)h.hlen + h.plen == F && chain_plausible(P, L, ss, q, unm, false) == 1u)
              L.best = (uint32_t)(q - ss);
          }
        }
      }
      __syncthreads();
      if (L.best != 0xFFFFFFFFu) {
        if (tid == 0) {
          L.aux0 = ss + L.best;
          stat_add(P, ST_P_LATTICE, 1);
        }
        break;
      }
    }
    scan_segment<G>(P, L, ss, tid, unm, !big);
    if (stats_on(P) && tid == 0) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      stat_add(P, ST_P_SCAN, t - tp);
      tp = t;
    }
    if (L.best != 0xFFFFFFFFu) {
      if (tid == 0) L.aux0 = ss + L.best;
      break;
    }
  }
  __syncthreads();
}

// Prologue of the run or piece at flat index `self` (whole workgroup): the
// entry scan of its range [rb, re), then lane 0 publishes (h, W, entry state,
// head frames) in its record and its entry granule. The chain state is left
// in L, the scanned segment in LDS (L.aux1), L.aux2 = W or NONE.
template <class G>
XYWS_DEV void prologue(const run_params& P, lds_t<G>& L, seg_io<G>& io, uint32_t tid, uint64_t self, uint64_t rb,
                       uint64_t re) {
  const uint64_t t0 = (stats_on(P) && tid == 0) ? __builtin_amdgcn_s_memtime() : 0;
  find_entry(P, L, io, tid, rb, re);
  const uint64_t tpub = (stats_on(P) && tid == 0) ? __builtin_amdgcn_s_memtime() : 0;
  if (tid == 0) {
    const uint64_t rng_end = re < P.hi ? re : NONE;
    const uint64_t q = L.aux0, ss = L.aux1;
    uint64_t h = NONE, W = NONE, hc = 0;
    cstate S;
    S.X = 0; S.cov_ps = 0; S.cov_start = 0; S.cov_kw = 0; S.cov_key = 0; S.st = S_NOCOV; S.pad = 0;
    if (q != NONE) {
      const hdr_info hq = hdr_at(P, L, ss, q, NONE);
      h = (hq.hlen == 2 || hq.hlen == 6) ? sat_add(q + hq.hlen, hq.plen) : q;
      const hdr_info hh = h < P.hi ? hdr_at(P, L, ss, h, NONE) : hq;
      if (h >= rng_end || h >= P.hi || !hh.hlen) {
        h = NONE;
      } else {
        W = (h + hh.hlen + 15) & ~15ull;
        // frames starting below W: parsed here, from bytes nobody writes yet
        S = frame_state(h, hh);
        hc = 1;
        record_start<G>(P, L, self, h);
        while (S.X < W && S.X < P.hi) {
          const hdr_info hx = hdr_at(P, L, ss, S.X, NONE);
          if (!hx.hlen) { S.st |= S_PARTIAL; break; }
          record_start<G>(P, L, self, S.X);
          S = frame_state(S.X, hx);
          hc++;
        }
      }
    }
    uint64_t* rec = P.rec + self * R_WORDS;
    st_store(rec + R_H, h);
    st_store(rec + R_W, W);
    put_state(rec + R_S0, S);
    st_store(rec + R_HEAD, hc);
    granule_store(P.flags + 2 * self, flag_published(L.E),
                  (h == NONE ? G_NONE : (h | ((W - h) << 46))) | granule_tag(L.E));
    L.S = S;
    L.cnt = hc;
    // dense-pass hint for the first segment: the entry's frame is small
    L.dense = (h != NONE && S.X - S.cov_start < 1024) ? G::FCAP : 0;
    L.aux2 = h == NONE ? NONE : W;
    stat_add(P, ST_RUNS, 1);
    if (h == NONE) stat_add(P, ST_NONE, 1);
    if (stats_on(P)) stat_add(P, ST_T_PRO, __builtin_amdgcn_s_memtime() - t0);
    if (stats_on(P)) stat_add(P, ST_P_PUB, __builtin_amdgcn_s_memtime() - tpub);
  }
  __syncthreads();
}

// The call's outputs (lane 0): frame count, total, carry out. cin: the
// incoming-carry snapshot (in LDS), o: the final chain state. The carry is
// assembled in 64-bit words (no byte array: nothing goes to scratch).
XYWS_DEV void write_outputs(const run_params& P, const xyws_carry* cin, uint64_t total, const cstate& o) {
  if (P.nframes) *P.nframes = total + P.tbias;  // (tbias: frames the lattice decoder decoded before a redirect)
  __hip_atomic_store(reinterpret_cast<uint64_t*>(P.head + 2), total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!P.cout) return;
  const uint64_t lo = P.lo, hi = P.hi;
  uint64_t pr = 0, ph = 0, key = 0, hl = 0, h0 = 0, h1 = 0;  // h0/h1: header bytes 0..7 / 8..13
  if (o.st & S_PARTIAL) {
    // the incomplete header: carried bytes (if still incomplete) + the batch tail
    const uint32_t c0 = (o.st & S_PARTCARRY) ? cin->hdr_len : 0u;
    const uint64_t from = (o.st & S_PARTCARRY) ? lo : o.X;
#pragma unroll
    for (uint32_t i = 0; i < XYWS_MAX_FRAME_HEADER_SIZE; i++) {
      uint64_t b = 0;
      bool have = true;
      if (i < c0) b = cin->hdr[i];
      else if (from + (i - c0) < hi) b = P.base[from + (i - c0)];
      else have = false;
      if (have && hl == i) {
        if (i < 8) h0 |= b << (8 * i); else h1 |= b << (8 * (i - 8));
        hl++;
      }
    }
  } else if (o.X > hi && !(o.st & S_NOCOV)) {
    if (o.st & S_CARRIED) {
      pr = cin->payload_remaining - (hi - lo);
      ph = cin->phase + (hi - lo);
      key = (uint64_t)cin->key[0] | ((uint64_t)cin->key[1] << 8) | ((uint64_t)cin->key[2] << 16) |
            ((uint64_t)cin->key[3] << 24);
    } else {
      const hdr_info hh = (o.st & S_HDRCARRY) ? header_carried(P, cin) : hdr_global(P, o.cov_start, NONE);
      pr = hh.plen - (hi - o.cov_ps);
      ph = hi - o.cov_ps;
      key = hh.key;
    }
  }
  // xyws_carry: payload_remaining, phase, frames_total, key[4] @24, hdr_len @28, hdr[14] @29
  uint64_t* c = reinterpret_cast<uint64_t*>(P.cout);
  c[0] = pr;
  c[1] = ph;
  c[2] = cin->frames_total + total;
  c[3] = key | (hl << 32) | (h0 << 40);
  c[4] = (h0 >> 24) | (h1 << 40);
  c[5] = h1 >> 24;
  c[6] = 0;
  c[7] = 0;
}

// finish_call's record scan (whole workgroup; every run has exited). When
// every run with an entry landed exactly on its successor's published entry
// (the usual case): frame counts, descriptor ordinals and the final state by a
// block-wide scan over the run records, no serial walk; L.act = 0, L.aux2 =
// the frame total, L.S = the final state. A run is good when its record is
// this call's, it did not give up on its successor, its chain landed on the
// successor's entry and that entry is the one the successor published;
// otherwise L.act = 1 (the serial walk repairs). One memory round trip when
// the runs fit one pass (every word loaded at once, the entries exchanged in
// LDS); tid 0 also loads the epoch and the incoming-carry snapshot (L.cinc).
// The entry of the run or piece at flat index f in this call, NONE when it has
// none: a piece exists only when its run agreed to the split (the run's
// R_SPLIT, written by this call's run: R_H of an unused piece is stale).
XYWS_DEV uint64_t entry_of(const run_params& P, uint64_t f) {
  // (both loads unconditional: no branch, no wait between them)
  const uint64_t h = st_load(P.rec + f * R_WORDS + R_H);
  const uint64_t sp = st_load(P.rec + (f & ~1ull) * R_WORDS + R_SPLIT);
  return ((f & 1) && sp == NONE) ? NONE : h;
}

template <class G>
XYWS_DEV void finish_fast(const run_params& P, lds_t<G>& L, uint32_t tid) {
  uint64_t* scr = reinterpret_cast<uint64_t*>(L.seg);  // scratch: wave totals
  // every run's entry, for the successor check (in LDS when it fits)
  constexpr bool HS_LDS = G::SEG >= 1024 + 16 * MAX_RUNS;
  uint64_t* hs = reinterpret_cast<uint64_t*>(L.seg + 1024);
  const bool one = HS_LDS && P.nflat <= G::NT;  // one pass: entries exchanged after the loads
  if (HS_LDS && !one) {
    for (uint32_t r = tid; r < P.nflat; r += G::NT) hs[r] = entry_of(P, r);
  }
  // this thread's record of the first pass: its loads go out together with
  // lane 0's epoch and carry loads (one memory round trip before the scan)
  struct rec_t {
    uint64_t h, cw, okw, ep, hn;
    cstate fs;
  };
  auto load_rec = [&](uint32_t r, rec_t& x) {
    const uint64_t* rec = P.rec + (uint64_t)r * R_WORDS;
    x.cw = st_load(rec + R_CNT);
    x.okw = st_load(rec + R_OK);
    x.ep = st_load(rec + R_EP);
    x.hn = st_load(rec + R_HN);
    x.fs = get_state(rec + R_F0);
    x.h = (HS_LDS && !one) ? hs[r] : entry_of(P, r);  // (last: the select waits for it)
  };
  // (every load goes out before the first LDS write or select that waits:
  // interleaved, each would wait for the ones before it)
  uint64_t c[9];
  if (tid == 0) {
    c[8] = st_load(reinterpret_cast<const uint64_t*>(P.head + HEAD_EPOCH));
#pragma unroll
    for (int i = 0; i < 8; i++) c[i] = st_load(reinterpret_cast<const uint64_t*>(P.cin) + i);
  }
  rec_t x0;
  x0.h = NONE; x0.cw = 0; x0.okw = OK_BIT; x0.ep = 0; x0.hn = NONE;
  if (tid < P.nflat) load_rec(tid, x0);
  if (tid == 0) {
    L.E = c[8] + 1;
#pragma unroll
    for (int i = 0; i < 8; i++) reinterpret_cast<uint64_t*>(&L.cinc)[i] = c[i];
  }
  __syncthreads();
  const uint64_t E = L.E;
  const uint32_t lane = tid & 63u, wave = tid >> 6;
  const bool plan = P.frames && P.cap;  // (the descriptor plan is read by k_stream_emit only)
  uint64_t carry = 0;
  uint32_t bad = 0, stale = 0, last = 0;
  bool has = false;
  cstate fsl;  // final state of this thread's last visible run
  for (uint32_t t0 = 0; t0 < P.nflat; t0 += G::NT) {
    const uint32_t r = t0 + tid;
    rec_t x;
    if (t0 == 0) {
      x = x0;
    } else {
      x.h = NONE; x.cw = 0; x.okw = OK_BIT; x.ep = E; x.hn = NONE;
      if (r < P.nflat) load_rec(r, x);
    }
    if (r >= P.nflat) x.ep = E;
    if (one) {
      if (r < P.nflat) hs[r] = x.h;
      __syncthreads();
    }
    const uint64_t h = x.h, okw = x.okw, ep = x.ep, hn = x.hn;
    const bool vis = r < P.nflat && (r == 0 || h != NONE);
    const uint64_t cnt = vis ? x.cw : 0;
    if (vis) {
      const uint64_t succ = okw >> 32;
      if (ep != E) stale = 1;
      if (!(okw & OK_BIT) || (okw & TMO_BIT) || ep != E) bad = 1;
      if (succ < P.nflat && hn != (HS_LDS ? hs[succ] : entry_of(P, succ))) bad = 1;
      last = r;
      fsl = x.fs;
      has = true;
    }
    uint64_t xs = cnt;  // wave inclusive scan
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(xs, o, 64);
      if (lane >= o) xs += y;
    }
    if (lane == 63) scr[wave] = xs;
    __syncthreads();
    uint64_t wb = 0, tot = 0;
    for (uint32_t w = 0; w < G::NT / 64; w++) {
      const uint64_t v = scr[w];
      if (w < wave) wb += v;
      tot += v;
    }
    if (vis && plan) {
      uint64_t* rw = P.rec + (uint64_t)r * R_WORDS;
      st_store(rw + R_EFROM, h);
      st_store(rw + R_ECNT, cnt);
      st_store(rw + R_EORD, carry + wb + xs - cnt);
      st_store(rw + R_ECARRY, r == 0 ? 1u : 0u);
    }
    carry += tot;
    __syncthreads();
  }
  // a record not written by this call: a run did not complete (reported; the
  // outputs of this call are invalid)
  if (__syncthreads_or(stale) && tid == 0) atomicOr(P.head + 1, 4u);
  const bool any_bad = __syncthreads_or(bad);
  if (tid == 0) L.aux1 = 0;
  __syncthreads();
  if (last) atomicMax(reinterpret_cast<unsigned long long*>(&L.aux1), (unsigned long long)last);
  __syncthreads();
  if (!any_bad) {
    if (tid == 0) L.aux2 = carry;
    if (has && last == L.aux1) L.S = fsl;
  }
  if (tid == 0) L.act = any_bad ? 1u : 0u;
  __syncthreads();
}

// Decode the run or piece at L.self after its prologue (whole workgroup): the
// chain from the entry state in L, writing from wlo (segment ss0, already in
// LDS when in_lds), then its results in its record. rng_end: the end of its
// range (NONE: the batch end); victim: it answers steal requests.
template <class G>
XYWS_DEV void decode_range(const run_params& P, lds_t<G>& L, seg_io<G>& io, uint32_t tid, uint64_t ss0, bool in_lds,
                           uint64_t wlo, uint64_t rng_end, bool victim) {
  if (tid == 0) {
    L.tail = 0; L.past = 0; L.ok = 0; L.done = 0; L.end = 0; L.tmo = 0; L.first_after = NONE;
    L.known = 0;
    // (the stride pass first, unless the previous call's frames were small and
    // irregular: a run of one or two segments would otherwise chase its first
    // segment serially -- one LDS round trip per frame -- before the dense
    // pass takes over from the second)
    L.sgood = P.dense0 ? 0u : 1u;
    L.rng_end = rng_end;
    L.victim = victim ? 1u : 0u;
    L.hn = NONE; L.Wn = NONE; L.succ = P.nflat;
    // (a run's own piece comes first when it is split while decoding)
    L.scan_j = L.self + 1;
  }
  __syncthreads();
  const uint64_t t1 = stats_on(P) ? __builtin_amdgcn_s_memtime() : 0;
  run_chain(P, L, io, tid, ss0, in_lds, wlo);
  if (tid == 0) {
    if (L.victim) {  // (the chain ended without a successor lookup)
      close_split(P, P.split + 2 * (L.self >> 1), L.E);
      L.victim = 0;
    }
    uint64_t* rec = P.rec + L.self * R_WORDS;
    const bool ok = !L.tmo && (L.succ >= P.nflat || (L.past && L.ok));
    st_store(rec + R_OK, (ok ? OK_BIT : 0) | (L.tmo ? TMO_BIT : 0) | ((uint64_t)L.succ << 32));
    st_store(rec + R_HN, L.hn);
    st_store(rec + R_WN, L.Wn);
    st_store(rec + R_CNT, L.cnt);
    st_store(rec + R_TAIL, L.tail);
    st_store(rec + R_FIRST, L.first_after);
    put_state(rec + R_F0, L.S);
    st_store(rec + R_EP, L.E);
    if (P.fst) st_store(rec + R_NREC, L.nrec);
    // what the workgroup finishing the call needs when every hand-over is
    // good: the frame total and the final state (the item without successor)
    uint64_t* hw = reinterpret_cast<uint64_t*>(P.head);
    if (!ok) __hip_atomic_fetch_or(hw + HW_BAD, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (L.cnt) __hip_atomic_fetch_add(hw + HW_TOTAL, L.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ok && L.succ >= P.nflat) put_state(hw + HW_FINAL, L.S);
    if (L.cnt) {
      const uint64_t fs = last_frame_size(L.S);
      fs_note(P, fs, fs);
    }
    if (stats_on(P)) st_store(rec + R_T2, __builtin_amdgcn_s_memrealtime());
    if (!ok) stat_add(P, ST_BAD, 1);
    if (L.tmo) stat_add(P, ST_GIVEUP, 1);
    stat_add(P, ST_FRAMES, L.cnt);
    if (stats_on(P)) stat_add(P, ST_T_MAIN, __builtin_amdgcn_s_memtime() - t1);
  }
  __syncthreads();
}

// A workgroup whose own run is done steals (whole workgroup): it asks the run
// with the most segments left (read from the runs' progress words) for the
// tail of its range. Returns the run that agreed (the piece starts at segment
// L.aux1 of its range), or NONE32 when no run has enough left.
template <class G>
XYWS_DEV uint32_t steal_piece(const run_params& P, lds_t<G>& L, uint32_t tid) {
  const uint64_t E = L.E;
  const uint64_t min_left = (P.opts & XYWS_OPT_TEST_STEAL) ? 3 : XYWS_STEAL_MIN_LEFT;
  for (uint32_t attempt = 0; attempt < 2 * P.nruns; attempt++) {
    if (tid == 0) L.aux0 = 0;
    __syncthreads();
    for (uint32_t r = tid; r < P.nruns; r += G::NT) {
      const uint64_t sw = st_load(P.split + 2 * r), pw = st_load(P.prog + r);
      if (split_is(sw, E, SP_FREE) && (pw >> 24) == (E & ((1ull << 40) - 1))) {
        const uint64_t rs = (uint64_t)r * P.rbytes;
        const uint64_t re = r + 1 < P.nruns ? rs + P.rbytes : P.hi;
        const uint64_t nseg = (re - rs + G::SEG - 1) / G::SEG, i = pw & 0xFFFFFFu;
        const uint64_t left = nseg > i + 1 ? nseg - i - 1 : 0;
        if (left >= min_left)
          atomicMax(reinterpret_cast<unsigned long long*>(&L.aux0), (unsigned long long)((left << 32) | (P.nruns - r)));
      }
    }
    __syncthreads();
    const uint64_t best = L.aux0;
    if (!best) return NONE32;
    const uint32_t v = P.nruns - (uint32_t)(best & 0xFFFFFFFFu);
    if (tid == 0) {
      L.act = 0;
      uint64_t* sw = P.split + 2 * (uint64_t)v;
      const unsigned long long fr = split_word(E, SP_FREE, 0);
      stat_add(P, ST_STEAL_REQ, 1);
      if (atomicCAS(reinterpret_cast<unsigned long long*>(sw), fr, (unsigned long long)split_word(E, SP_REQ, 0)) == fr) {
        // the run answers within a segment or two (it polls every segment)
        uint32_t it = 0;
        uint64_t w = split_word(E, SP_REQ, 0);
        while (split_is(w, E, SP_REQ) && it < SPIN) {
          __builtin_amdgcn_s_sleep(2);
          w = st_load(sw);
          it++;
        }
        if (split_is(w, E, SP_ACC)) {
          L.act = 1;
          L.aux1 = split_seg(w);
        } else if (split_is(w, E, SP_REQ)) {
          atomicOr(P.head + 1, 2u);  // (bounded wait timed out: reported, the run is left alone)
        }
      }
    }
    __syncthreads();
    if (L.act) return v;
  }
  return NONE32;
}

// ---------------------------------------------------------------- kernels
// One workgroup per run (ticket order). After its own run a workgroup takes
// pieces of slower runs (steal_piece) until none is worth taking; the run /
// piece loop keeps one copy of the prologue and of the chain in the kernel.
template <class G>
__device__ __attribute__((always_inline)) inline void finish_call(run_params P, lds_t<G>& L, uint32_t tid);

template <class G>
__global__ void __launch_bounds__(G::NT, G::WPE) k_stream_runs(run_params P0) {
  extern __shared__ __attribute__((aligned(16))) uint8_t xs_lds[];
  lds_t<G>& L = *reinterpret_cast<lds_t<G>*>(xs_lds);
  // after the lattice decoder: nothing left, the rest of the batch, or all of it
  run_params P = P0;
  if (!lat_redirect(P)) return;
  const uint32_t tid0 = threadIdx.x, tid = tid0;
  if (tid == 0) {
    L.ticket = atomicAdd(P.head, 1u);
    L.E = st_load(reinterpret_cast<const uint64_t*>(P.head + HEAD_EPOCH)) + 1;
  }
  __syncthreads();
  const uint32_t run = uniform32(L.ticket);
  if (run >= P.nruns) return;
  const bool steal = (P.opts & (XYWS_OPT_STEAL | XYWS_OPT_TEST_STEAL)) != 0;
  {
    const uint64_t rs = (uint64_t)run * P.rbytes;
    uint64_t* rec = P.rec + 2 * (uint64_t)run * R_WORDS;
    if (tid == 0) {
      // no descriptors unless finish_call plans them (the run and its piece)
      st_store(rec + R_ECNT, 0);
      st_store(rec + R_WORDS + R_ECNT, 0);
      st_store(rec + R_SPLIT, NONE);
      // the run can be asked for the tail of its range from now on
      st_store(P.split + 2 * (uint64_t)run, split_word(L.E, steal ? SP_FREE : SP_CLS, 0));
      L.split_poll[0] = split_word(L.E, SP_FREE, 0);
      L.split_e = NONE;
      L.self = 2 * (uint64_t)run;
      L.rs = rs;
      if (stats_on(P)) {
        st_store(rec + R_T0, __builtin_amdgcn_s_memrealtime());
        // HW_REG_XCC_ID (hwreg 20), bits [3:0]
        st_store(rec + R_XCC, (uint64_t)(__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xFu));
      }
      if (run == 0) {
        // snapshot of the incoming carry for finish_call / k_stream_emit
        // (the caller's carry may alias the carry out, which finish writes)
        // (in words, through LDS: no private copy)
        const xyws_carry* cu = P.cin_user ? P.cin_user : &k_zero_carry;
        uint64_t cw[8];
#pragma unroll
        for (int i = 0; i < 8; i++) cw[i] = reinterpret_cast<const uint64_t*>(cu)[i];
        // (sc1 stores: another CU's finish reads them)
#pragma unroll
        for (int i = 0; i < 8; i++) {
          reinterpret_cast<uint64_t*>(&L.cinc)[i] = cw[i];
          st_store(reinterpret_cast<uint64_t*>(P.cin) + i, cw[i]);
        }
        uint64_t c0;
        L.S = initial_state(P, &L.cinc, c0);
        L.cnt = c0;
        // dense-pass hint for the first segment, as a prologue sets it: the
        // frame at the first boundary is small (run 0 chased its first
        // segment serially before: the slowest run of a small-frame batch)
        {
          const hdr_info h0 = (L.S.st & S_PARTIAL) ? hdr_info{} : hdr_global(P, L.S.X, NONE);
          L.dense = (h0.hlen && h0.plen + h0.hlen < 1024) ? G::FCAP : 0;
        }
        st_store(rec + R_H, P.lo);
        st_store(rec + R_W, P.lo);
        put_state(rec + R_S0, L.S);
        st_store(rec + R_HEAD, c0);
        granule_store(P.flags, flag_published(L.E), P.lo | granule_tag(L.E));
      } else {
        // claim the own prologue (a predecessor that finds it unclaimed gives
        // up on this run instead of waiting for a workgroup that may not be
        // running)
        granule_store(P.flags + 4 * (uint64_t)run, flag_claimed(L.E), 0);
      }
      // the item decoded first: the own run
      L.ib = rs;
      L.ie = rs + P.rbytes;
      // (test mode: every fourth run starts late, so that others finish first
      // and take pieces of it whatever the hardware's own imbalance)
      if ((P.opts & XYWS_OPT_TEST_STEAL) && (run & 3u) == 1u)
        for (int i = 0; i < 24; i++) __builtin_amdgcn_s_sleep(127);
    }
  }
  __syncthreads();
  for (;;) {
    seg_io<G> io;  // (per item: no prefetch registers live across the steal)
    // (an opaque copy of the lane index per item: hipcc would otherwise hoist
    // the lane address math of the chain out of this loop and spill in it)
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint64_t self = uniform64(L.self);
    const bool own = !(self & 1);
    const uint64_t rb = uniform64(L.ib), re = uniform64(L.ie);
    const uint64_t rng_end = re < P.hi ? re : NONE;
    uint64_t wlo = P.lo, ss0 = 0;
    bool in_lds = false, entry = true;
    if (tid == 0) L.nrec = 0;  // (read by lane 0 after the barriers below)
    if (self != 0) {
      prologue<G>(P, L, io, tid, self, rb, re);
      entry = L.aux2 != NONE;  // (no entry: the chain of an earlier run covers this range)
      wlo = uniform64(L.aux2);
      // the chain starts in the scanned segment (usual) or on the grid after it
      const uint64_t a1 = uniform64(L.aux1);
      ss0 = a1 + (wlo - a1) / G::SEG * G::SEG;
      in_lds = ss0 == a1;
      // (the next segment's loads were issued before the scan)
      if (entry && in_lds && ss0 + G::SEG < P.hi && io.pf != ss0 + G::SEG) io.issue(P, ss0 + G::SEG, tid);
    }
    if (tid == 0 && stats_on(P)) st_store(P.rec + self * R_WORDS + R_T1, __builtin_amdgcn_s_memrealtime());
    if (entry) {
      decode_range<G>(P, L, io, tid, ss0, in_lds, wlo, rng_end, own && steal);
      if (tid == 0 && own) st_store(P.rec + self * R_WORDS + R_SPLIT, L.split_e);
    } else if (tid == 0 && own) {
      close_split(P, P.split + self, L.E);
    }
    if (!steal) break;
    // the next item: a piece of a slower run
    const uint32_t v = steal_piece<G>(P, L, tid);
    if (v == NONE32) break;
    if (tid == 0) {
      const uint64_t vs = (uint64_t)v * P.rbytes;
      L.self = 2 * (uint64_t)v + 1;
      L.ib = vs + L.aux1 * G::SEG;
      L.ie = v + 1 < P.nruns ? vs + P.rbytes : P.hi;
      L.rs = L.ib;
      L.split_e = NONE;
      if (stats_on(P)) st_store(P.rec + L.self * R_WORDS + R_T0, __builtin_amdgcn_s_memrealtime());
    }
    __syncthreads();
  }
  // End of the workgroup: one done-count add; the workgroup whose add comes
  // last finishes the call (no second kernel on the stream). The finisher may
  // read payload bytes other workgroups stored (the repair walk's undo re-XORs
  // a mis-speculated run's bytes, possibly stored on another XCD, whose L2 is
  // not coherent with this one), so the hand-off is the producer/consumer form
  // of MI355X_MICROARCH.md §Workgroup dispatch: every storing wave drains its
  // stores, a workgroup barrier, an agent-scope release (L2 write-back) and
  // the add; the finisher takes an agent-scope acquire before it reads.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid0 == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the flag must not overtake the write-back)
    const uint32_t last = atomicAdd(P.head + 2 * HW_DONE, 1u) + 1 == P.nruns ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    L.act = last;
  }
  __syncthreads();
  if (L.act) finish_call<G>(P, L, tid0);
}

// The next run or piece after flat index r with an entry (lane 0; every
// prologue is published by now), or nflat.
XYWS_DEV uint64_t next_visible(const run_params& P, uint64_t r) {
  for (uint64_t j = r + 1; j < P.nflat; j++)
    if (entry_of(P, j) != NONE) return j;
  return P.nflat;
}

// The piece of run r as its workgroup recorded it (lane 0). Its hand-over is
// good only if its record is this call's and its successor's published entry
// is the one its chain landed on.
XYWS_DEV void load_piece(const run_params& P, walk_t& w, uint64_t r) {
  const uint64_t* rec = P.rec + r * R_WORDS;
  const uint64_t okw = st_load(rec + R_OK);
  w.r = r;
  w.efrom = st_load(rec + R_H);
  w.ecarry = r == 0 ? 1u : 0u;
  w.cnt = st_load(rec + R_CNT);
  w.tail = st_load(rec + R_TAIL);
  w.first = st_load(rec + R_FIRST);
  w.F = get_state(rec + R_F0);
  w.wlim = st_load(rec + R_WN);
  w.succ = okw >> 32;
  w.tmo = (okw & TMO_BIT) ? 1u : 0u;
  w.ok = (okw & OK_BIT) ? 1u : 0u;
  if (w.ok && w.succ < P.nflat && st_load(rec + R_HN) != entry_of(P, w.succ)) w.ok = 0;
}

// Set up a chase from state S with the given successor limits (lane 0).
template <class G>
XYWS_DEV void chain_start(lds_t<G>& L, const cstate& S, uint64_t hn, uint64_t Wn, uint64_t succ) {
  L.S = S;
  L.S.st &= ~S_CUT;
  L.hn = hn; L.Wn = Wn; L.succ = succ;
  L.known = 1; L.cnt = 0; L.tail = 0; L.past = 0; L.ok = 0; L.done = 0; L.end = 0; L.dense = 0; L.tmo = 0;
  L.sgood = 1;
  L.first_after = NONE;
  L.best = 0;
  L.rng_end = NONE;
  L.victim = 0;
}

// Walk the runs from run 0 along their successors, repairing every boundary
// whose chain did not land on the successor's entry, then the frame count, the
// carry and the descriptor plan (one workgroup; every run has exited).
// Serial walk with repairs (whole workgroup; finish_call runs it when the
// fast path found a bad hand-over). Lane 0 keeps the current chain piece in
// L.wk: the run whose descriptor plan it fills (r, efrom, ecarry), its frames
// (cnt; tail = those past the successor's entry), its final state F, its
// write limit, and how it hands over (ok / tmo / succ).
//  * tmo (the run gave up on a successor that had not started): bridge from
//    F, writing from the write limit, up to the next run with an entry; the
//    bridge's frames join the piece.
//  * !ok (the chain missed the successor's entry): undo the successor's run
//    (replaying its own chain: XOR is an involution and a chain never writes
//    its own header bytes), redo it from F, writing from the write limit; the
//    redo is the next piece.
//  * ok: the successor's own record is the next piece.
template <class G>
XYWS_DEV void finish_walk(const run_params& P, lds_t<G>& L, uint32_t tid) {
  seg_io<G> io;
  if (tid == 0) {
    L.aux2 = 0;
    load_piece(P, L.wk, 0);
  }
  __syncthreads();
  for (uint32_t guard = 0; guard <= 4 * P.nflat + 4; guard++) {
    if (tid == 0) {
      walk_t& w = L.wk;
      if (w.tmo) {
        const uint64_t sj = next_visible(P, w.r);
        w.succ = sj;
        w.act = 4;
        stat_add(P, ST_BRIDGE, 1);
        chain_start(L, w.F, sj < P.nflat ? st_load(P.rec + sj * R_WORDS + R_H) : NONE,
                    sj < P.nflat ? st_load(P.rec + sj * R_WORDS + R_W) : NONE, sj);
      } else {
        uint64_t* rec = P.rec + w.r * R_WORDS;
        st_store(rec + R_EFROM, w.efrom);
        st_store(rec + R_ECNT, w.cnt);
        st_store(rec + R_EORD, L.aux2);
        st_store(rec + R_ECARRY, w.ecarry);
        L.aux2 += w.cnt;
        if (w.succ >= P.nflat) {
          w.act = 0;  // done
          L.S = w.F;
        } else if (w.ok) {
          w.act = 1;  // next run as recorded
          load_piece(P, w, w.succ);
        } else {
          stat_add(P, ST_REPAIR, 1);
          w.act = 2;
          const uint64_t* rs = P.rec + w.succ * R_WORDS;
          chain_start(L, get_state(rs + R_S0), st_load(rs + R_HN), st_load(rs + R_WN), st_load(rs + R_OK) >> 32);
        }
      }
    }
    __syncthreads();
    const uint32_t act = L.wk.act;
    if (act == 0) break;
    if (act == 1) continue;
    if (act == 4) {
      // bridge: the chain from where the run stopped to the next entry
      const uint64_t wp = L.wk.wlim;
      io.pf = NONE;
      run_chain(P, L, io, tid, wp & ~15ull, false, wp);
      __threadfence();
      __syncthreads();
      if (tid == 0) {
        walk_t& w = L.wk;
        w.cnt += L.cnt;
        w.tail = L.tail;
        w.first = L.first_after;
        w.F = L.S;
        w.ok = w.succ >= P.nflat || (L.past && L.ok);
        w.wlim = L.Wn;
        w.tmo = 0;
      }
      __syncthreads();
      continue;
    }
    // act == 2: undo the successor's run exactly as it ran
    const uint64_t sj = L.wk.succ;
    const uint64_t* rs = P.rec + sj * R_WORDS;
    const uint64_t W = st_load(rs + R_W);
    const uint64_t hn = L.hn, Wn = L.Wn, succ = L.succ;
    io.pf = NONE;
    run_chain(P, L, io, tid, W & ~15ull, false, W);
    __threadfence();  // the undo's stores are visible to the redo's loads
    __syncthreads();
    // redo from the exact state, same successor, from our write limit
    const uint64_t wp = L.wk.wlim;
    if (tid == 0) {
      chain_start(L, L.wk.F, hn, Wn, succ);
    }
    __syncthreads();
    io.pf = NONE;
    run_chain(P, L, io, tid, wp & ~15ull, false, wp);
    __threadfence();
    __syncthreads();
    if (tid == 0) {
      walk_t& w = L.wk;
      const uint64_t ws = st_load(rs + R_OK);
      w.efrom = w.first != NONE ? w.first : w.F.X;
      w.cnt = w.tail + L.cnt;
      w.r = sj;
      w.ecarry = 0;
      w.tail = L.tail;
      w.first = L.first_after;
      w.F = L.S;
      w.succ = L.succ;
      w.tmo = (ws & TMO_BIT) ? 1u : 0u;
      w.ok = !w.tmo && (L.succ >= P.nflat || (L.past && L.ok));
      w.wlim = L.Wn;
    }
    __syncthreads();
  }
}

// Walk the runs from run 0 along their successors, repairing every boundary
// whose chain did not land on the successor's entry, then the frame count, the
// carry and the descriptor plan (one workgroup; every run has exited).
// Run by the workgroup whose done-count add came last (every other workgroup
// has written its records and exited). When every hand-over was good and no
// descriptors are asked for, the call's outputs come from the end-of-call
// words (the frame total, the final state): a few loads. Otherwise the run
// records are scanned (finish_fast: total, carry, descriptor plan, bad
// hand-overs) and bad hand-overs are repaired (finish_walk). Then the ticket,
// the done count and the end-of-call words are reset and the epoch advances,
// so the next call (or graph replay) starts clean without a memset.
// (inlined: as a call it cost ~900 B of private segment per lane for the
// call frame; inlined the decode loop still spills nothing, checked in the
// ISA, and the private segment is ~190 B, in the prologue and this path)
template <class G>
__device__ __attribute__((always_inline)) inline void finish_call(run_params P, lds_t<G>& L, uint32_t tid) {
  uint64_t* hw = reinterpret_cast<uint64_t*>(P.head);
  if (tid == 0) {
    const uint64_t bad = st_load(hw + HW_BAD);
    L.act = (bad || (P.frames && P.cap)) ? 1u : 0u;
  }
  __syncthreads();
  bool walked = false;
  if (L.act) {
    finish_fast<G>(P, L, tid);
    walked = L.act != 0;
    if (walked) finish_walk<G>(P, L, tid);
    if (tid == 0) write_outputs(P, &L.cinc, L.aux2, L.S);
  } else if (tid == 0) {
    // (all loads first: one memory round trip)
    uint64_t c[8];
#pragma unroll
    for (int i = 0; i < 8; i++) c[i] = st_load(reinterpret_cast<const uint64_t*>(P.cin) + i);
    const uint64_t total = st_load(hw + HW_TOTAL);
    const cstate S = get_state(hw + HW_FINAL);
#pragma unroll
    for (int i = 0; i < 8; i++) reinterpret_cast<uint64_t*>(&L.cinc)[i] = c[i];
    write_outputs(P, &L.cinc, total, S);
  }
  if (tid == 0) {
    if (P.fst) {
      // the frame-start lists stand unless they overflowed or a repair changed
      // the plan (k_stream_emit then re-walks the chains)
      st_store(hw + HW_EMIT_FLAG, (walked || st_load(hw + HW_EMIT_SLOW)) ? 1u : 0u);
      st_store(hw + HW_EMIT_SLOW, 0);
    }
    pol_publish(P, L.E, G::NT == 512 ? DEC_RUNS512 : DEC_RUNS);
    st_store(hw + HW_BAD, 0);
    st_store(hw + HW_TOTAL, 0);
    st_store(hw + HW_DONE, 0);
    // the ticket starts the next call at zero; the epoch word advances (this
    // call's entry granules read as stale from now on)
    __hip_atomic_store(P.head, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    st_store(reinterpret_cast<uint64_t*>(P.head + HEAD_EPOCH), L.E);
  }
}

XYWS_DEV void write_frame(const run_params& P, uint64_t ord, uint64_t start, const hdr_info& h,
                          uint64_t ps, int32_t hdr_shift) {
  xyws_frame f;
  f.frame_off = (int64_t)(start - P.lo + P.obias) - hdr_shift;
  f.payload_off = (int64_t)(ps - P.lo + P.obias);
  f.payload_len = h.plen;
  f.key[0] = (uint8_t)h.key; f.key[1] = (uint8_t)(h.key >> 8);
  f.key[2] = (uint8_t)(h.key >> 16); f.key[3] = (uint8_t)(h.key >> 24);
  f.flags = h.flags;
  f.hdr_len = (uint8_t)h.hlen;
  f.status = (uint8_t)(h.status | (sat_add(ps, h.plen) > P.hi ? XYWS_ST_PAYLOAD_INCOMPLETE : 0));
  f.reserved = 0;
  P.frames[ord] = f;
}

// Descriptors, one workgroup per run or piece at the ordinals finish_call
// planned: the carried-header frame first (run 0), then the frame starts the
// item recorded, in chain order, each header parsed from memory by its own lane (headers are never modified by the decode). When those lists are
// unusable (HW_EMIT_FLAG) lane 0 re-chases the item's frames from its first one.
__global__ void __launch_bounds__(256) k_stream_emit(run_params P0) {
  run_params P = P0;
  if (!lat_redirect(P)) return;
  const uint32_t r = blockIdx.x, tid = threadIdx.x;
  if (r >= P.nflat) return;
  const uint64_t* rec = P.rec + (uint64_t)r * R_WORDS;
  const uint64_t ord = st_load(rec + R_EORD);
  const uint64_t n = st_load(rec + R_ECNT);
  if (n == 0 || ord >= P.cap) return;
  const uint64_t end = ord + n < P.cap ? ord + n : P.cap;
  const bool ecarry = st_load(rec + R_ECARRY) != 0;
  const bool slow = st_load(reinterpret_cast<const uint64_t*>(P.head) + HW_EMIT_FLAG) != 0;
  uint64_t o = ord, X = st_load(rec + R_EFROM);
  if (ecarry) {  // run 0: the carried-header frame comes first
    X = P.lo;
    if (!P.cin->payload_remaining && P.cin->hdr_len) {
      const hdr_info hh = header_carried(P, P.cin);
      if (hh.hlen) {
        const uint64_t ps = P.lo + (hh.hlen - P.cin->hdr_len);
        if (tid == 0) write_frame(P, o, P.lo, hh, ps, (int32_t)P.cin->hdr_len);
        o++;
        X = sat_add(ps, hh.plen);
      }
    } else if (P.cin->payload_remaining) {
      X = sat_add(P.lo, P.cin->payload_remaining);
    }
  }
  if (slow) {
    if (tid != 0) return;
    while (o < end && X < P.hi) {
      const hdr_info hh = hdr_global(P, X, NONE);
      if (!hh.hlen) break;
      const uint64_t ps = X + hh.hlen;
      write_frame(P, o++, X, hh, ps, 0);
      X = sat_add(ps, hh.plen);
    }
    return;
  }
  const uint64_t k = st_load(rec + R_NREC);
  const uint64_t* src = P.fst + (uint64_t)r * P.rcap;
  for (uint64_t i = tid; i < k && o + i < end; i += 256) {
    const uint64_t x = src[i];
    const hdr_info hh = hdr_global(P, x, NONE);
    write_frame(P, o + i, x, hh, x + hh.hlen, 0);
  }
}

// Empty batch: the state passes through unchanged.
__global__ void k_stream_empty(const xyws_carry* cin, xyws_carry* cout, uint64_t* nframes) {
  if (threadIdx.x) return;
  if (nframes) *nframes = 0;
  if (cout) {
    xyws_carry c;
    if (cin) c = *cin;
    else for (int i = 0; i < 64; i++) reinterpret_cast<uint8_t*>(&c)[i] = 0;
    *cout = c;
  }
}

#include "xyws_lattice.h"

constexpr uint64_t HEAD_BYTES = 1024;  // u32 [0] ticket, [1] error, [2..3] total, [4..5] epoch; bytes [64..128) carry,
                                       // [128..512) stats, [512..576) end-of-call words (HW_*)

// hipFuncSetAttribute applies to the current device: once per (device,
// geometry), under a lock (one process may drive several devices from several
// threads).
template <class G>
int set_lds_attr() {
  static std::mutex mu;
  static bool done[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return XYWS_ERR_HIP;
  std::lock_guard<std::mutex> lk(mu);
  if (done[dev]) return XYWS_OK;
  const int lds = (int)sizeof(lds_t<G>);
  if (hipFuncSetAttribute((const void*)k_stream_runs<G>, hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
      hipSuccess)
    return XYWS_ERR_HIP;
  done[dev] = true;
  return XYWS_OK;
}

template <class G>
int launch_runs(const run_params& P, hipStream_t stream) {
  const size_t lds = sizeof(lds_t<G>);
  if (const int rc = set_lds_attr<G>()) return rc;
  hipLaunchKernelGGL(k_stream_runs<G>, dim3(P.nruns), dim3(G::NT), lds, stream, P);
  if (P.frames && P.cap) hipLaunchKernelGGL(k_stream_emit, dim3(P.nflat), dim3(256), 0, stream, P);
  return hipGetLastError() == hipSuccess ? XYWS_OK : XYWS_ERR_HIP;
}

}  // namespace

void stream_scratch_init(stream_scratch* s, int device) {
  s->mem = nullptr;
  s->bytes = 0;
  s->max_runs = 0;
  s->fmem = nullptr;
  s->fbytes = 0;
  s->ncu = 256;
  s->pol_h = nullptr;
  s->pol_d = nullptr;
  s->lmem = nullptr;
  s->lmax_segs = 0;
  void* ph = nullptr;
  if (hipHostMalloc(&ph, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
    void* pd = nullptr;
    memset(ph, 0, 64);
    if (hipHostGetDevicePointer(&pd, ph, 0) == hipSuccess) {
      s->pol_h = static_cast<volatile uint64_t*>(ph);
      s->pol_d = static_cast<uint64_t*>(pd);
    } else {
      (void)hipHostFree(ph);
    }
  }
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && n > 0)
    s->ncu = n;
}

void stream_scratch_free(stream_scratch* s) {
  if (s->pol_h) (void)hipHostFree(const_cast<uint64_t*>(s->pol_h));
  s->pol_h = nullptr;
  s->pol_d = nullptr;
  if (s->lmem) (void)hipFree(s->lmem);
  s->lmem = nullptr;
  s->lmax_segs = 0;
  if (s->mem) (void)hipFree(s->mem);
  if (s->fmem) (void)hipFree(s->fmem);
  s->mem = nullptr;
  s->bytes = 0;
  s->max_runs = 0;
  s->fmem = nullptr;
  s->fbytes = 0;
}

// Frame-start lists for descriptor emission: one region per flat item of
// twice the caller's capacity spread over the runs + 1024 (a region that
// overflows switches the call to the chain re-walk). Grown on demand, not
// under graph capture (xyws_ctx_reserve).
static uint64_t region_entries(uint64_t cap, uint64_t nruns) { return 2 * ((cap + nruns - 1) / nruns) + 1024; }
static int fmem_grow(stream_scratch* s, uint64_t bytes, bool capturing) {
  if (s->fmem && bytes <= s->fbytes) return XYWS_OK;
  if (capturing) return XYWS_ERR_CAPACITY;
  void* m = nullptr;
  if (hipMalloc(&m, bytes) != hipSuccess) return XYWS_ERR_NOMEM;
  if (s->fmem) {
    (void)hipDeviceSynchronize();
    (void)hipFree(s->fmem);
  }
  s->fmem = m;
  s->fbytes = bytes;
  return XYWS_OK;
}

// Scratch layout for up to `runs` runs (2 * runs flat indices):
//   head | entry granules (16 B per flat index) | split words (16 B per run) |
//   progress words (8 B per run) | records (R_WORDS x 8 B per flat index)
// Everything up to the records is zeroed at allocation (epoch 0: stale).
static uint64_t granules_bytes(uint64_t runs) { return (32 * runs + 255) & ~255ull; }
static uint64_t split_bytes(uint64_t runs) { return (16 * runs + 255) & ~255ull; }
static uint64_t prog_bytes(uint64_t runs) { return (8 * runs + 255) & ~255ull; }
static uint64_t records_off(uint64_t runs) {
  return HEAD_BYTES + granules_bytes(runs) + split_bytes(runs) + prog_bytes(runs);
}

static int scratch_grow(stream_scratch* s, uint64_t runs) {
  if (s->mem && runs <= s->max_runs) return XYWS_OK;
  const uint64_t want = runs < 64 ? 64 : runs;
  const uint64_t bytes = records_off(want) + 2 * want * R_WORDS * 8;
  void* m = nullptr;
  if (hipMalloc(&m, bytes) != hipSuccess) return XYWS_ERR_NOMEM;
  if (s->mem) {
    (void)hipDeviceSynchronize();
    (void)hipFree(s->mem);
  }
  s->mem = m;
  s->bytes = bytes;
  s->max_runs = want;
  return xyws_internal::zero_now(m, records_off(want)) == hipSuccess ? XYWS_OK : XYWS_ERR_HIP;
}

// Lattice decoder scratch for up to `segs` segments: LW_STAT words of
// scratch and one result word per segment, all zeroed at allocation (epoch 0:
// no result of any call).
static uint64_t lat_max_grid(const stream_scratch* s) {
  const uint64_t g = (uint64_t)s->ncu;  // (one workgroup per CU)
  return g > 64 ? g : 64;
}
static int lat_grow(stream_scratch* s, uint64_t segs, bool capturing) {
  if (s->lmem && segs <= s->lmax_segs) return XYWS_OK;
  if (capturing) return XYWS_ERR_CAPACITY;
  const uint64_t want = segs < 64 ? 64 : segs;
  // (statuses, group counts, LW_BRK replicas, one list per workgroup)
  const uint64_t bytes = 8 * (lat_sl_off(want) + lat_max_grid(s) * LAT_LSW);
  void* m = nullptr;
  if (hipMalloc(&m, bytes) != hipSuccess) return XYWS_ERR_NOMEM;
  if (s->lmem) {
    (void)hipDeviceSynchronize();
    (void)hipFree(s->lmem);
  }
  s->lmem = m;
  s->lmax_segs = want;
  return xyws_internal::zero_now(m, bytes) == hipSuccess ? XYWS_OK : XYWS_ERR_HIP;
}

int stream_scratch_unmask_counter(stream_scratch* s, bool capturing, uint32_t** out) {
  if (const int rc = lat_grow(s, 1, capturing)) return rc;
  *out = reinterpret_cast<uint32_t*>(static_cast<uint64_t*>(s->lmem) + LW_UNMASK);
  return XYWS_OK;
}

// The most runs any production geometry launches: four per CU (G_MID, the
// echo-sized batches), capped at MAX_RUNS.
static uint64_t max_prod_runs(const stream_scratch* s) {
  const uint64_t r = (uint64_t)s->ncu * 4;
  return r < MAX_RUNS ? r : MAX_RUNS;
}

int stream_scratch_reserve_frames(stream_scratch* s, uint64_t max_batch_bytes, uint64_t max_frames) {
  // the descriptor regions total 8 * 2R * (2 * cap / R + 1024 + 4) bytes:
  // largest at the most runs a production geometry launches
  const uint64_t runs = max_prod_runs(s);
  (void)max_batch_bytes;
  const uint64_t nflat = 2 * runs;
  // (any smaller run count gives regions whose total is no larger, up to the
  // rounding of cap / runs: + 4 entries per item)
  return fmem_grow(s, 8 * nflat * (region_entries(max_frames, runs) + 4), false);
}

int stream_scratch_reserve(stream_scratch* s, uint64_t max_batch_bytes) {
  // the production geometries (stream_decode_fused): one run per segment up
  // to their run count (1, 2 or 4 per CU on 128, 64 or 16 KiB segments); the
  // small-segment test mode grows scratch lazily
  uint64_t runs = 0;
  const uint64_t segs[3] = {G_PROD::SEG, G_PROD2::SEG, G_MID::SEG}, per_cu[3] = {1, 2, 4};
  for (int g = 0; g < 3; g++) {
    const uint64_t nseg = (max_batch_bytes + 15 + segs[g] - 1) / segs[g];
    const uint64_t r = (uint64_t)s->ncu * per_cu[g], maxr = r < MAX_RUNS ? r : MAX_RUNS;
    const uint64_t n = nseg < maxr ? nseg : maxr;
    if (n > runs) runs = n;
  }
  if (const int rc = scratch_grow(s, runs)) return rc;
  // the lattice decoder's (production geometries: the 75 KiB segments have the most)
  return lat_grow(s, (max_batch_bytes + 15 + G_LAT5::SEG - 1) / G_LAT5::SEG, false);
}

int stream_scratch_stats(stream_scratch* s, uint64_t out[XYWS_NSTATS]) {
  if (!s->mem) return XYWS_ERR_INVALID;
  if (hipDeviceSynchronize() != hipSuccess) return XYWS_ERR_HIP;
  return hipMemcpy(out, static_cast<uint8_t*>(s->mem) + 128, 8 * XYWS_NSTATS, hipMemcpyDeviceToHost) == hipSuccess
             ? XYWS_OK : XYWS_ERR_HIP;
}

int stream_scratch_lattice(stream_scratch* s, uint64_t out[5]) {
  for (int i = 0; i < 5; i++) out[i] = 0;
  if (hipDeviceSynchronize() != hipSuccess) return XYWS_ERR_HIP;
  if (s->mem && hipMemcpy(out, static_cast<uint8_t*>(s->mem) + 8 * HW_DPOL, 8, hipMemcpyDeviceToHost) != hipSuccess)
    return XYWS_ERR_HIP;
  if (s->lmem) {
    const uint32_t w[4] = {LW_NBAIL_POL, LW_NBAIL_HYP, LW_NLOOP_A, LW_NLOOP_B};
    for (int i = 0; i < 4; i++)
      if (hipMemcpy(out + 1 + i, static_cast<uint64_t*>(s->lmem) + w[i], 8, hipMemcpyDeviceToHost) != hipSuccess)
        return XYWS_ERR_HIP;
  }
  return XYWS_OK;
}

int64_t stream_scratch_records(stream_scratch* s, uint64_t* out, uint64_t max_recs) {
  if (!s->mem) return XYWS_ERR_INVALID;
  if (hipDeviceSynchronize() != hipSuccess) return XYWS_ERR_HIP;
  const uint64_t n = max_recs < 2 * s->max_runs ? max_recs : 2 * s->max_runs;
  const uint8_t* rec = static_cast<const uint8_t*>(s->mem) + records_off(s->max_runs);
  return hipMemcpy(out, rec, n * R_WORDS * 8, hipMemcpyDeviceToHost) == hipSuccess ? (int64_t)n : XYWS_ERR_HIP;
}

uint32_t stream_scratch_error(stream_scratch* s, bool clear) {
  if (!s->mem) return 0;
  uint32_t v[2] = {0, 0};
  if (hipMemcpy(v, s->mem, 8, hipMemcpyDeviceToHost) != hipSuccess) return 0xFFFFFFFFu;
  if (clear && v[1] && xyws_internal::zero_now(static_cast<uint8_t*>(s->mem) + 4, 4) != hipSuccess) return 0xFFFFFFFFu;
  return v[1];
}

// The run decoder's geometry, by the same statistics: regular frames under
// WG512_MAX_FRAME take two 512-thread workgroups per CU on 64 KiB segments
// (while one workgroup chases its segment, the other's stores drain: c2's
// 264-byte frames 0.247 -> 0.181 ms, same box), the rest one 1024-thread
// workgroup on 128 KiB segments (c1's 4 KiB frames 0.152 vs 0.158 ms; c4's
// mixed sizes up to 1 MiB 0.496 vs 1.19).
// Small frames of mixed sizes take it too when the batch is small (under one
// 128 KiB segment per CU: the default geometry would give each run one
// segment, and a run's latency is the call's): echo-sized batches of 0-1000 B
// frames 115-135 -> 72-79 us per call (profiles/r03z_echo_geometry.txt).
constexpr uint64_t WG512_MAX_FRAME = 2048;
// Echo-sized batches (under 32 KiB per CU) of small frames of mixed sizes:
// four 256-thread workgroups per CU on 16 KiB segments, four times the runs
// of the 512-thread geometry (a run's latency is the call's: 4 MiB of 0-1000 B
// frames with descriptors 80.6 -> 65.7 us, 1 MiB 81.9 -> 57.4; 8 KiB segments
// 78.9 / 53.6; at 16 MiB the 512-thread geometry stays faster, 94 vs 125).
static bool mid_preferred(const stream_scratch* s, uint64_t len) {
  if (!s->pol_h) return false;
  const uint64_t fsmin = s->pol_h[2], fsmax = s->pol_h[3];
  return fsmax && fsmax < WG512_MAX_FRAME && fsmin != fsmax && len <= (uint64_t)s->ncu * 32768;
}
constexpr uint64_t DENSE0_MAX_FRAME = 2048;
constexpr uint64_t BIGSCAN_MIN_FRAME = 16384;
static bool wg512_preferred(const stream_scratch* s, uint64_t len) {
  if (!s->pol_h) return false;
  const uint64_t fsmin = s->pol_h[2], fsmax = s->pol_h[3];
  const bool small_batch = len < (uint64_t)s->ncu * G_PROD::SEG;
  return fsmax && fsmax < WG512_MAX_FRAME && (fsmin == fsmax || small_batch);
}

// The lattice decoder (xyws_lattice.h) goes first when the previous call on
// this stream found frames of one size, at least LAT_FMIN bytes (the policy
// words; the bench batches c1/c2/c3/c5 and every batch of one message size),
// or when there was no previous call; the run decoder follows it in the same
// stream (XYWS_OPT_REDIRECT) and decodes what it left: nothing (it exits at
// once), the batch from the first frame off the lattice, or all of it. Its
// miss costs its loads of the batch's first segments.
static bool lattice_preferred(const stream_scratch* s) {
  if (!s->pol_h) return false;
  const uint64_t fsmin = s->pol_h[2], fsmax = s->pol_h[3];
  if (!s->pol_h[0]) return true;  // (no call has finished on this stream)
  return fsmax && fsmin == fsmax && fsmin >= LAT_FMIN;
}

template <class GA, class GB>
int launch_lattice(const run_params& P, uint32_t grid, hipStream_t stream) {
  static std::mutex mu;
  static bool done[64] = {};
  using LL = lat_lds<llay<GA, GB>>;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return XYWS_ERR_HIP;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (!done[dev]) {
      if (hipFuncSetAttribute((const void*)k_stream_lattice<GA, GB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sizeof(LL)) != hipSuccess)
        return XYWS_ERR_HIP;
      done[dev] = true;
    }
  }
  hipLaunchKernelGGL((k_stream_lattice<GA, GB>), dim3(grid), dim3(GB::NT), sizeof(LL), stream, P);
  return hipGetLastError() == hipSuccess ? XYWS_OK : XYWS_ERR_HIP;
}

int stream_decode_fused(stream_scratch* s, uint8_t* base, uint64_t lo, uint64_t hi,
                        const xyws_carry* cin, xyws_carry* cout, xyws_frame* frames, uint64_t cap,
                        uint64_t* nframes, uint32_t opts, hipStream_t stream) {
  opts &= ~XYWS_OPT_REDIRECT;  // (set here only)
  if (hi == lo) {
    hipLaunchKernelGGL(k_stream_empty, dim3(1), dim3(64), 0, stream, cin, cout, nframes);
    return hipGetLastError() == hipSuccess ? XYWS_OK : XYWS_ERR_HIP;
  }
  const bool small = (opts & XYWS_OPT_SMALL_SEG) != 0;
  constexpr uint32_t RUN_MODES = XYWS_OPT_PARSE_ONLY | XYWS_OPT_WG512 | XYWS_OPT_DIAG | XYWS_OPT_TEST_GIVEUP |
                                 XYWS_OPT_STEAL | XYWS_OPT_TEST_STEAL | XYWS_OPT_RUNS | XYWS_OPT_NO_LATTICE |
                                 XYWS_OPT_RUNS_NOWAIT | XYWS_OPT_WG1024 | XYWS_OPT_NO_LATENTRY;
  const bool want_lat = !(opts & (RUN_MODES | XYWS_OPT_NO_LATDEC)) &&
                        ((opts & XYWS_OPT_LATTICE) || (!small && lattice_preferred(s)));
  const bool mid = !small && !(opts & (XYWS_OPT_WG512 | XYWS_OPT_WG1024)) &&
                   ((opts & XYWS_OPT_WG256) || mid_preferred(s, hi - lo));
  const bool wg512 = !small && !mid && !(opts & XYWS_OPT_WG1024) && ((opts & XYWS_OPT_WG512) || wg512_preferred(s, hi - lo));
  const uint64_t seg = small ? G_SMALL::SEG : mid ? G_MID::SEG : wg512 ? G_PROD2::SEG : G_PROD::SEG;
  // Runs get equal byte ranges (multiples of 16, one segment at least): every
  // workgroup streams the same number of bytes, and a run whose chain crosses
  // into the next range loads only the bytes below the successor's W there.
  const uint64_t nseg = (hi + seg - 1) / seg;
  uint64_t nruns, rbytes;
  const uint64_t r = small ? nseg : (uint64_t)s->ncu * (mid ? 4u : wg512 ? 2u : 1u);
  const uint64_t maxr = r < MAX_RUNS ? r : MAX_RUNS;
  if (nseg <= maxr) {
    rbytes = seg;
  } else {
    rbytes = ((hi + maxr - 1) / maxr + 15) & ~15ull;
  }
  nruns = (hi + rbytes - 1) / rbytes;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(stream, &cs);
  if (nruns > s->max_runs || !s->mem) {
    if (cs != hipStreamCaptureStatusNone) return XYWS_ERR_CAPACITY;
    const int rc = scratch_grow(s, nruns);
    if (rc) return rc;
  }
  uint8_t* m = static_cast<uint8_t*>(s->mem);
  run_params P;
  P.base = base; P.lo = lo; P.hi = hi; P.rbytes = rbytes;
  P.nruns = (uint32_t)nruns;
  P.cout = cout; P.frames = frames; P.cap = cap; P.nframes = nframes;
  P.head = reinterpret_cast<uint32_t*>(m);
  P.nflat = 2 * P.nruns;
  P.flags = reinterpret_cast<uint64_t*>(m + HEAD_BYTES);
  P.split = reinterpret_cast<uint64_t*>(m + HEAD_BYTES + granules_bytes(s->max_runs));
  P.prog = reinterpret_cast<uint64_t*>(m + HEAD_BYTES + granules_bytes(s->max_runs) + split_bytes(s->max_runs));
  P.rec = reinterpret_cast<uint64_t*>(m + records_off(s->max_runs));
  P.opts = opts;
  // The ticket is zero here (zeroed at allocation, reset by finish_call
  // after every call); granules, split and progress words carry the epoch of
  // the call that wrote them; the error word [1] is sticky until read back.
  // Run 0 snapshots the incoming carry into scratch.
  if ((opts & XYWS_OPT_STATS) && hipMemsetAsync(m + 128, 0, 8 * XYWS_NSTATS, stream) != hipSuccess) return XYWS_ERR_HIP;
  P.cin_user = cin;
  P.cin = reinterpret_cast<xyws_carry*>(m + 64);
  P.fst = nullptr; P.rcap = 0;
  P.pol = s->pol_d;
  P.lat = static_cast<uint64_t*>(s->lmem);  // (nullable: the device policy word's second copy)
  P.segb = (uint32_t)seg;
  P.tbias = 0;
  P.obias = 0;
  P.nseg = 0;
  // the lattice entry (find_entry): the previous call's frames all F bytes
  // long, several per segment
  P.pfs = 0;
  P.dense0 = 0;
  if (s->pol_h && !(opts & XYWS_OPT_NO_LATENTRY)) {
    const uint64_t fsmin = s->pol_h[2], fsmax = s->pol_h[3];
    if (fsmax && fsmin == fsmax && fsmax <= seg / 4) P.pfs = fsmax;
  }
  // small frames of mixed sizes last call (every run's last frame under
  // DENSE0_MAX_FRAME, not all one size): the dense pass from each run's first
  // segment (echo-sized batches of 0-1000 B frames: one segment per run)
  if (s->pol_h && !(opts & XYWS_OPT_NO_DENSE0)) {
    const uint64_t fsmin = s->pol_h[2], fsmax = s->pol_h[3];
    if (fsmax && fsmin != fsmax && fsmax < DENSE0_MAX_FRAME) P.dense0 = 1;
  }
  // large frames of mixed sizes last call (some last frame of BIGSCAN_MIN_FRAME
  // or more: config 4): the entry scans filter a whole segment in one pass (a
  // range start usually lies inside a large frame: the first 16 KiB hold no
  // entry, and their own round of checks cost 3.6 us per scanned segment, c4)
  P.bigscan = (opts & XYWS_OPT_BIGSCAN) ? 1u : 0u;
  if (s->pol_h && !(opts & XYWS_OPT_NO_BIGSCAN)) {
    const uint64_t fsmin = s->pol_h[2], fsmax = s->pol_h[3];
    if (fsmax && fsmin != fsmax && fsmax >= BIGSCAN_MIN_FRAME) P.bigscan = 1;
  }
  if (frames && cap) {
    const uint64_t rc_n = region_entries(cap, nruns);
    const int rc = fmem_grow(s, 8 * (uint64_t)P.nflat * rc_n, cs != hipStreamCaptureStatusNone);
    if (rc) return rc;
    P.fst = static_cast<uint64_t*>(s->fmem);
    P.rcap = rc_n;
  }
  if (want_lat) {
    // the lattice decoder first; the run decoder after it reads its redirect
    // record. Its segment geometry (75 KiB for frames of LAT5_MIN_FRAME and
    // more, else 120 KiB), the first-segment gate and its bail-out after an
    // irregular call are decided in the kernel (the batch's first frame, the
    // device policy word HW_DPOL); the grid covers the smaller segments.
    const uint64_t lseg = small ? G_LAT_SMALL::SEG : G_LAT5::SEG;
    const uint64_t lnseg = (hi + lseg - 1) / lseg;
    if (const int rc = lat_grow(s, lnseg, cs != hipStreamCaptureStatusNone)) return rc;
    run_params PL = P;
    PL.opts &= ~XYWS_OPT_LAT_NOGATE;
    PL.lat = static_cast<uint64_t*>(s->lmem);
    PL.lgrp = PL.lat + LW_STAT + s->lmax_segs;
    PL.lbrk = PL.lat + lat_rep_off(s->lmax_segs);
    PL.lsl = PL.lat + lat_sl_off(s->lmax_segs);
    PL.nseg = lnseg;  // (the kernel counts the segments of the geometry it takes)
    const uint64_t maxg = small ? 64 : (uint64_t)s->ncu;
    const uint32_t grid = (uint32_t)(lnseg < maxg ? lnseg : maxg);
    const int rc = small ? launch_lattice<G_LAT_SMALL, G_LAT_SMALL>(PL, grid, stream)
                         : launch_lattice<G_LAT5, G_LAT>(PL, grid, stream);
    if (rc) return rc;
    P.lat = PL.lat;
    P.opts |= XYWS_OPT_REDIRECT;
    if (opts & XYWS_OPT_LATX_ONLY) return XYWS_OK;  // (timing experiment: the lattice kernel alone)
  }
  return small ? launch_runs<G_SMALL>(P, stream)
         : mid   ? launch_runs<G_MID>(P, stream)
         : wg512 ? launch_runs<G_PROD2>(P, stream)
                 : launch_runs<G_PROD>(P, stream);
}
