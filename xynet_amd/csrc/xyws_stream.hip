// xyws_stream.hip — fused single-pass stream decoder for gfx950 (default mode of
// xyws_decode_stream).
//
// Problem: in a back-to-back batch the start of frame k+1 is known only after
// the header of frame k is parsed (websocket_frame_header.h:305-385 gives the
// header size and the payload length), so frame boundaries form a linked list
// through the batch. A serial chase from HBM costs one dependent load per
// frame; a separate index pass would read the batch twice. This kernel reads
// every byte once and keeps it in registers until its frames are known.
//
// Geometry: a SEGMENT is 64 KiB owned by one 256-thread workgroup; lane t
// holds 16 chunks of 16 B (chunk k at segment offset (k*256 + t)*16, so each
// load instruction of a wave covers 1 KiB contiguously) = 64 VGPRs, loaded and
// stored through a per-segment buffer descriptor (base and range in SGPRs, one
// 32-bit offset per lane). Two workgroups fit per CU (VGPRs <= 256, LDS ~62
// KiB each): while one resolves boundaries the other streams. (128 KiB
// segments, 128 data VGPRs, spilled: the resolution code needs the rest.) Segments are handed out by an atomic ticket,
// so every segment a workgroup waits on is owned by a running workgroup
// (forward progress with no co-residency assumption).
//
// Per segment:
//  1. Issue all 16 loads. For each 32 KiB sub-tile: copy it (+16 B halo) to
//     LDS, SWAR-prefilter every byte position for a plausible client header
//     (RSV = 0, known opcode, MASK set), fully parse the candidates (minimal
//     length form, control-frame rules, frame fits the batch, successor inside
//     the sub-tile is itself a candidate) and append the survivors, in
//     position order, to a segment-wide survivor list.
//  2. Link survivors (successor = survivor at pos + H + len, or EXIT past the
//     segment) and walk the graph once (memoized): every node learns its
//     outcome (which exit it reaches), its remaining frame count, and — on the
//     first walk that reached each outcome — its ordinal along that walk.
//     Speculation over a 64 KiB span is strong: a false candidate must chain
//     through plausible headers all the way out of the segment.
//  3. Publish the AGGREGATE record: the first 8 exiting nodes (position,
//     outcome, remaining count) and up to 4 outcomes (exit, last frame).
//  4. Decoupled look-back: the nearest INCLUSIVE predecessor gives an exact
//     state; it is carried through later segments with their aggregates (the
//     exact entry must be one of their published nodes, or lie past them), or
//     we wait for that segment's own inclusive record. After resolving its own
//     segment a workgroup keeps HELPING: it carries the exact state forward
//     through successors whose aggregates are already published and publishes
//     their inclusive records, so the frontier runs ahead of the data.
//  5. The exact in-segment chain from the true entry: the suffix of a primary
//     walk (parallel, by ordinal) or an exact header chase in global memory
//     (header bytes are never modified, so any workgroup may read them).
//  6. XOR every register chunk with the rotated keys of the frames covering it
//     and store the changed chunks.
// Speculation only decides speed; correctness rests on the exact state of
// step 4 and the exact chain of step 5, so any byte stream (RSV bits, reserved
// opcodes, unmasked or non-minimal frames) decodes as the reference parses it.
//
// Inter-workgroup hand-off follows MI355X_MICROARCH.md §Workgroup dispatch
// (table row 1): record words are written with agent-scope (sc1) stores by ONE
// lane, drained with s_waitcnt vmcnt(0), then an sc1 flag store; readers poll
// the flag with sc1 loads and read the record with sc1 loads. Flags and the
// ticket are zeroed by hipMemsetAsync before every launch. Every spin is
// bounded and reports through the device error word.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xyws_stream.h"
#include "xyws_device.h"

namespace {

constexpr uint32_t SEG = 65536;          // segment bytes (per workgroup)
constexpr uint32_t SUB = 32768;          // sub-tile bytes staged in LDS
constexpr uint32_t NSUB = SEG / SUB;     // 2
constexpr uint32_t NT = 256;             // threads per workgroup
constexpr uint32_t CHS = SEG / (16 * NT);  // 32 chunks per lane
constexpr uint32_t CHSUB = SUB / (16 * NT);  // 8 chunks per lane per sub-tile
constexpr uint32_t HALO = 16;
constexpr uint32_t SMAX = 512;           // survivors tracked per segment
constexpr uint32_t LV = 9;               // jump-table levels: 2^LV >= SMAX
constexpr uint32_t FCAP = SUB / 16;      // frame-list entries per pass (overlays the sub-tile)
constexpr uint32_t NENT = 16;            // aggregate entry nodes (2 per record word)
constexpr uint32_t NOUT = 8;             // aggregate outcomes (2 record words each)
constexpr uint32_t SPIN = 1u << 24;      // bounded spins (~1 s)

constexpr uint32_t WIN = 64;             // segments seen by one look-back (one per lane)
constexpr uint32_t BKT = 8;              // exits kept per target segment during speculation
constexpr uint16_t N_EXIT = 0xFFFF, N_DEAD = 0xFFFE;
constexpr uint8_t O_DEAD = 0xFE, O_UNREC = 0xFD;  // node outcome marks
constexpr uint16_t J_TERM = 0xFFFF;      // jump past the end of a chain
constexpr uint16_t T_DEAD = 0xFFFF;      // chain ends in a dead end

// composition-state bits
constexpr uint32_t S_PARTIAL = 1;    // stream ended in an incomplete header at X
constexpr uint32_t S_NOCOV = 2;      // no frame covers the bytes before X
constexpr uint32_t S_CARRIED = 4;    // covering frame = the open frame carried in
constexpr uint32_t S_HDRCARRY = 8;   // covering frame's header began in the previous batch
constexpr uint32_t S_PARTCARRY = 16; // the carried partial header is still incomplete
constexpr uint32_t S_KEEP = S_NOCOV | S_CARRIED | S_HDRCARRY;

// record layout: 64 x u64 per segment
enum {
  R_META = 0,              // n_entries | n_outcomes << 8 | overflow << 16
  R_ENT0 = 1,              // NENT entries, two per word: pos (16) | rem (13) << 16 | outcome (3) << 29
  R_OUT0 = 9,              // NOUT outcomes x 2 words: exit; cov_ps - ss (20) | hlen (4) << 20 | kw << 32
  R_CI = 25,               // assumed input state  (X, cov_ps, cov_start, kw | st << 32)
  R_CO = 29,               // output state computed from it
  R_CN = 33,               // frames whose header starts in the segment (given the input)
  R_EX = 34,               // exact output from the slow path (4 words)
  R_EN = 38,               // exact frame count from the slow path
  R_NA = 39,               // frame count aggregate (exact)
  R_NI = 40,               // inclusive frame-count prefix
  R_WORDS = 64
};

struct fent {
  uint32_t start, ps, end, kw;  // segment-relative; ps/end clamped to [0, 2^32-1]
};

struct cstate {
  uint64_t X;          // first frame start >= current position (absolute)
  uint64_t cov_ps;     // payload start of the frame ending at X
  uint64_t cov_start;  // header start of that frame
  uint64_t cnt;        // frames whose header completed before X
  uint32_t cov_kw;     // aligned key word of that frame
  uint32_t st;         // S_* bits
};

struct __attribute__((aligned(16))) st_lds {
  union {
    uint8_t sub[SUB + HALO];  // pass 1: sub-tile bytes
    fent flist[FCAP];         // pass 2: frame list
  };
  uint64_t bits[SUB / 64];    // candidate bitmap of the current sub-tile
  uint32_t s_pos[SMAX];       // survivor position (segment-relative)
  uint32_t s_nrel[SMAX];      // successor position (segment-relative, saturating)
  uint32_t s_key[SMAX];
  uint16_t s_nxt[SMAX];       // successor survivor index / N_EXIT / N_DEAD
  uint16_t s_jmp[LV][SMAX];   // s_jmp[b][i]: the 2^b-th successor of i (J_TERM past the chain end)
  uint16_t s_rem[SMAX];       // frames from this node to the chain end
  uint16_t s_last[SMAX];      // last node of the chain (T_DEAD: ends in a dead end)
  uint8_t s_out[SMAX];        // outcome id / O_* mark
  uint8_t s_hlen[SMAX];
  uint32_t scan[8];
  // broadcast scalars
  uint64_t seg_id;
  uint32_t nsurv, overflow, nfl, pass_done;
  cstate in, out;
  uint64_t chase_X, fbase;
  uint32_t mode, node_x, rem_x, nent_pub, nout_pub, more_j;
  uint64_t outs[NOUT][4];     // aggregate outcomes: exit, cov_ps, cov_start, kw
  uint32_t ents[NENT];        // aggregate entries (packed as in the record)
  uint32_t bk_n[WIN];         // speculation: exits landing in each window segment
  uint32_t bk[WIN][BKT];
  uint64_t nbase;             // frame ordinal of this segment's first frame
};

struct st_params {
  uint8_t* base;
  uint64_t lo, hi, nseg;
  const xyws_carry* cin;  // private snapshot of the incoming carry
  xyws_carry* cout;
  xyws_frame* frames;
  uint64_t cap;
  uint64_t* nframes;
  uint32_t* head;   // [0] ticket, [1] error word, [2] finished segments, [4..5] u64 frame total
  uint32_t* fA;     // per segment: aggregate published
  uint32_t* fC;     // per segment: (assumed input, output) published
  uint32_t* fV;     // per segment: 1 = output exact (validated), 2 = exact via the slow path
  uint32_t* fN;     // per segment: 1 = count aggregate, 2 = inclusive count prefix
  uint32_t* fP;     // per segment: 1 = assumed input == predecessor's published output, 2 = not
  uint64_t* recs;   // R_WORDS per segment
  uint32_t opts;
};

// ---------------------------------------------------------------- debug counters
// With XYWS_OPT_STATS the kernel counts resolution events into head[16..32)
// (read back by xyws_debug_stats). Off by default: one uniform branch each.
enum { ST_EXACT_IN = 0, ST_SPEC, ST_NOSPEC, ST_VALID, ST_SLOW, ST_RECOMP, ST_NOANCHOR,
       ST_MODE1, ST_MODE2, ST_NSURV, ST_SPINS,
       ST_T_PASS1 = 16, ST_T_WALK, ST_T_INPUT, ST_T_CHAIN, ST_T_VALID, ST_T_COUNT, ST_T_XOR, ST_T_STORE,
       ST_NSTAT = 32 };

// ---------------------------------------------------------------- hand-off
XYWS_DEV void st_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
XYWS_DEV uint64_t st_load(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
XYWS_DEV uint32_t flag_load(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
XYWS_DEV void flag_publish(uint32_t* p, uint32_t v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // record stores drained before the flag
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
XYWS_DEV bool stat_on(const st_params& P) { return (P.opts & XYWS_OPT_STATS) != 0; }
XYWS_DEV void stat_add(const st_params& P, uint32_t i, uint64_t v) {
  if (__builtin_amdgcn_mbcnt_lo(~0u, 0) == 0)  // one lane
    atomicAdd(reinterpret_cast<unsigned long long*>(P.head + 32) + i, (unsigned long long)v);
}
// Per-phase cycle accounting (stats builds only): adds now - *t to slot i.
XYWS_DEV void stat_phase(const st_params& P, uint32_t i, uint64_t& t) {
  if (!stat_on(P)) return;
  const uint64_t now = __builtin_amdgcn_s_memtime();
  stat_add(P, i, now - t);
  t = now;
}

XYWS_DEV bool wid0(uint32_t wave) { return wave == 0; }

XYWS_DEV bool flag_wait(const uint32_t* p, uint32_t want, uint32_t* err) {
  for (uint32_t it = 0; it < SPIN; it++) {
    if (flag_load(p) >= want) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      return true;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  atomicOr(err, 2u);
  return false;
}

// ---------------------------------------------------------------- parsing
// Header at absolute position p from global memory (header bytes are never
// written by this kernel). With a carried partial header (h0 > 0) the first h0
// bytes come from `pre`.
// Header from 16 little-endian bytes held in four dwords w[0..3] (byte i =
// w[i/4] >> 8*(i%4)), of which `avail` are valid. Same semantics as
// parse_header_bytes (websocket_frame_header.h:305-385).
XYWS_DEV hdr_info parse_header_words(const uint32_t w[4], uint32_t avail) {
  hdr_info h;
  h.plen = 0; h.key = 0; h.hlen = 0; h.flags = 0; h.status = 0;
  if (avail < 2) return h;
  const uint32_t b0 = w[0] & 0xFF, b1 = (w[0] >> 8) & 0xFF;
  const uint32_t l7 = b1 & 0x7Fu;
  const uint32_t ext = l7 == 126 ? 2u : (l7 == 127 ? 8u : 0u);
  const uint32_t masked = b1 >> 7;
  const uint32_t need = 2u + ext + 4u * masked;
  if (avail < need) return h;
  // bytes 2..9 as a big-endian length; bytes k..k+3 as the key (k = 2 + ext)
  const uint64_t lo8 = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  const uint64_t hi8 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  const uint64_t b2_9 = (lo8 >> 16) | (hi8 << 48);  // bytes 2..9, little-endian
  uint64_t len = l7;
  if (ext == 2) len = ((b2_9 & 0xFF) << 8) | ((b2_9 >> 8) & 0xFF);
  else if (ext == 8) len = __builtin_bswap64(b2_9);
  uint32_t key = 0;
  if (masked) {
    const uint32_t k = 2 + ext;  // 2, 4 or 10
    key = (k == 2) ? __builtin_amdgcn_alignbyte(w[1], w[0], 2)
        : (k == 4) ? w[1] : __builtin_amdgcn_alignbyte(w[3], w[2], 2);
  }
  const uint32_t op = b0 & 0x0Fu;
  uint8_t st = 0;
  if (b0 & 0x70u) st |= XYWS_ST_RSV;
  if ((op >= 3 && op <= 7) || op >= 11) st |= XYWS_ST_RESERVED_OPCODE;
  if ((l7 == 126 && len < 126) || (l7 == 127 && len <= 0xFFFFull)) st |= XYWS_ST_NONMINIMAL_LENGTH;
  if (l7 == 127 && (len >> 63)) st |= XYWS_ST_LENGTH_MSB;
  if (op >= 8 && (!(b0 & 0x80u) || len > 125)) st |= XYWS_ST_BAD_CONTROL;
  if (!masked) st |= XYWS_ST_UNMASKED;
  h.plen = len;
  h.key = key;
  h.hlen = need;
  h.flags = (uint8_t)(op | ((b0 & 0x80u) ? XYWS_FLAG_FIN : 0u) | (masked ? XYWS_FLAG_HAS_MASK : 0u));
  h.status = st;
  return h;
}

// Four dwords starting at byte address p (any alignment): aligned dword loads
// (never one that starts at or beyond `limit`) + byte-align funnel shifts.
XYWS_DEV void load16_global(const uint8_t* base, uint64_t p, uint64_t limit, uint32_t w[4]) {
  const uint64_t a = p & ~3ull;
  const uint32_t sh = (uint32_t)(p & 3);
  uint32_t r[5];
#pragma unroll
  for (int i = 0; i < 5; i++)
    r[i] = (a + 4 * i < limit) ? *reinterpret_cast<const uint32_t*>(base + a + 4 * i) : 0u;
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
}

XYWS_DEV hdr_info header_global(const uint8_t* base, uint64_t p, uint64_t hi) {
  uint32_t w[4];
  load16_global(base, p, hi, w);
  const uint64_t room = hi > p ? hi - p : 0;
  return parse_header_words(w, room < 16 ? (uint32_t)room : 16u);
}

// Header whose first h0 bytes were carried from the previous batch.
XYWS_DEV hdr_info header_carried(const uint8_t* base, uint64_t lo, uint64_t hi, const xyws_carry* c) {
  uint8_t hb[XYWS_MAX_FRAME_HEADER_SIZE];
  const uint32_t h0 = c->hdr_len < XYWS_MAX_FRAME_HEADER_SIZE ? c->hdr_len : XYWS_MAX_FRAME_HEADER_SIZE;
  uint32_t n = 0;
  for (; n < h0; n++) hb[n] = c->hdr[n];
  for (; n < XYWS_MAX_FRAME_HEADER_SIZE && lo + (n - h0) < hi; n++) hb[n] = base[lo + (n - h0)];
  return parse_header_bytes(hb, n);
}

XYWS_DEV hdr_info header_lds(const uint8_t* sub, uint32_t prel, uint64_t pabs, uint64_t hi) {
  const uint32_t a = prel & ~3u, sh = prel & 3u;
  const uint32_t* q = reinterpret_cast<const uint32_t*>(sub + a);
  uint32_t w[4];
  const uint32_t r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
  w[0] = __builtin_amdgcn_alignbyte(r1, r0, sh);
  w[1] = __builtin_amdgcn_alignbyte(r2, r1, sh);
  w[2] = __builtin_amdgcn_alignbyte(r3, r2, sh);
  w[3] = __builtin_amdgcn_alignbyte(r4, r3, sh);
  const uint64_t room = hi > pabs ? hi - pabs : 0;
  return parse_header_words(w, room < 16 ? (uint32_t)room : 16u);
}

// Conformance filter of a fully parsed header (speculation only).
XYWS_DEV bool plausible(const hdr_info& h, uint8_t b1) {
  if (!h.hlen) return false;
  const uint32_t op = h.flags & 0x0F;
  if (op >= 8 && (!(h.flags & XYWS_FLAG_FIN) || h.plen > 125)) return false;
  const uint32_t l7 = b1 & 0x7F;
  if (l7 == 126 && h.plen < 126) return false;
  if (l7 == 127 && (h.plen <= 0xFFFF || (h.plen >> 62))) return false;
  return true;
}

XYWS_DEV uint32_t clamp_rel(uint64_t x, uint64_t ts) {
  if (x <= ts) return 0;
  const uint64_t d = x - ts;
  return d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
}

// State before the first byte of the batch (the "inclusive record of segment
// -1"), from the carry snapshot.
XYWS_DEV cstate initial_state(const st_params& P) {
  cstate s;
  s.X = P.lo; s.cov_ps = P.lo; s.cov_start = P.lo; s.cnt = 0; s.cov_kw = 0; s.st = S_NOCOV;
  const xyws_carry* c = P.cin;
  const uint64_t R = c->payload_remaining;
  if (R) {
    const uint32_t k = (uint32_t)c->key[0] | ((uint32_t)c->key[1] << 8) |
                       ((uint32_t)c->key[2] << 16) | ((uint32_t)c->key[3] << 24);
    s.X = sat_add(P.lo, R);
    s.cov_ps = P.lo;
    s.cov_kw = aligned_key(k, P.lo, c->phase);
    s.st = S_CARRIED;
    return s;
  }
  const uint32_t h0 = c->hdr_len;
  if (h0) {
    hdr_info h = header_carried(P.base, P.lo, P.hi, c);
    if (!h.hlen) {  // still incomplete: the whole batch belongs to the header
      s.st = S_NOCOV | S_PARTIAL | S_PARTCARRY;
      return s;
    }
    s.cov_start = P.lo;
    s.cov_ps = P.lo + (h.hlen - h0);
    s.X = sat_add(s.cov_ps, h.plen);
    s.cov_kw = aligned_key(h.key, s.cov_ps, 0);
    s.cnt = 1;
    s.st = S_HDRCARRY;
  }
  return s;
}

XYWS_DEV cstate load_state(const uint64_t* r) {
  cstate s;
  uint64_t w[4];
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = st_load(r + i);
  s.X = w[0]; s.cov_ps = w[1]; s.cov_start = w[2];
  s.cov_kw = (uint32_t)w[3]; s.st = (uint32_t)(w[3] >> 32); s.cnt = 0;
  return s;
}

XYWS_DEV void store_state(uint64_t* r, const cstate& s) {
  st_store(r + 0, s.X);
  st_store(r + 1, s.cov_ps);
  st_store(r + 2, s.cov_start);
  st_store(r + 3, (uint64_t)s.cov_kw | ((uint64_t)s.st << 32));
}

XYWS_DEV bool same_state(const cstate& a, const cstate& b) {
  return a.X == b.X && a.cov_ps == b.cov_ps && a.cov_start == b.cov_start &&
         a.cov_kw == b.cov_kw && a.st == b.st;
}

// Exact output state of segment j (fV[j] = fv >= 1); j < 0: the batch start.
XYWS_DEV cstate exact_out(const st_params& P, int64_t j, uint32_t fv) {
  if (j < 0) return initial_state(P);
  return load_state(P.recs + (uint64_t)j * R_WORDS + (fv == 2 ? R_EX : R_CO));
}

// Exact chase by header reads in global memory from s.X while s.X < lim.
XYWS_DEV void chase_global(const st_params& P, cstate& s, uint64_t lim, uint32_t max_hops,
                           bool* incomplete) {
  const uint64_t stop = lim < P.hi ? lim : P.hi;
  for (uint32_t hop = 0; hop < max_hops; hop++) {
    if ((s.st & S_PARTIAL) || s.X >= stop) return;
    hdr_info h = header_global(P.base, s.X, P.hi);
    if (!h.hlen) { s.st = (s.st & S_KEEP) | S_PARTIAL; return; }
    s.cov_start = s.X;
    s.cov_ps = s.X + h.hlen;
    s.cov_kw = aligned_key(h.key, s.cov_ps, 0);
    s.X = sat_add(s.cov_ps, h.plen);
    s.cnt++;
    s.st = 0;
  }
  if (!(s.st & S_PARTIAL) && s.X < stop) *incomplete = true;
}

// ---------------------------------------------------------------- resolution
XYWS_DEV uint32_t rl32(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
XYWS_DEV uint64_t rl64(uint64_t v, uint32_t l) {
  return ((uint64_t)rl32((uint32_t)(v >> 32), l) << 32) | rl32((uint32_t)v, l);
}
XYWS_DEV uint32_t bp32(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src * 4), (int)v);
}
XYWS_DEV uint64_t bp64(uint64_t v, uint32_t src) {
  return ((uint64_t)bp32((uint32_t)(v >> 32), src) << 32) | bp32((uint32_t)v, src);
}
XYWS_DEV cstate bcast_state(const cstate& s) {  // lane 0's state to every lane
  cstate r;
  r.X = rl64(s.X, 0); r.cov_ps = rl64(s.cov_ps, 0); r.cov_start = rl64(s.cov_start, 0);
  r.cnt = rl64(s.cnt, 0); r.cov_kw = rl32(s.cov_kw, 0); r.st = rl32(s.st, 0);
  return r;
}
XYWS_DEV void wave_sync() {  // order this wave's LDS accesses across lanes
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

constexpr uint32_t S_NONE = 0x80000000u;  // "no speculation available" marker in cstate.st

// Step A: the input state of segment k as the whole wave sees it.
//  exact: the nearest validated predecessor's output already reaches k
//         (every segment between it and k is covered by its last frame);
//  else : speculation from the aggregates of the 63 preceding segments: an
//         entry node is trusted when some outcome of an earlier segment (or
//         the exact anchor) exits exactly onto it ("link support"); k takes
//         the trusted outcome of the nearest segment that reaches it.
XYWS_DEV cstate resolve_input(const st_params& P, st_lds& L, uint64_t k, uint32_t lane, bool& exact) {
  exact = false;
  if (k == 0) { exact = true; return initial_state(P); }
  const uint64_t ts = k * SEG;
  // A1: nearest predecessor with an exact output (j = -1: the batch start)
  const int64_t j = (int64_t)k - 1 - (int64_t)lane;
  const uint32_t fv = j >= 0 ? flag_load(P.fV + j) : (j == -1 ? 3u : 0u);
  const uint64_t mv = __ballot(fv >= 1);
  cstate E;
  int64_t a = -2;
  if (mv) {
    const uint32_t l = (uint32_t)__builtin_ctzll(mv);
    a = (int64_t)k - 1 - (int64_t)l;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    E = exact_out(P, a, rl32(fv, l));
    if ((E.st & S_PARTIAL) || E.X >= ts) { exact = true; E.cnt = 0; return E; }
  }
  // A2: speculation over the window [k-63, k] (lane l = segment k-63+l)
  const int64_t w0 = (int64_t)k - (int64_t)(WIN - 1);
  const int64_t g = w0 + (int64_t)lane;
  // every window segment was ticketed before k and publishes its aggregate
  // from local work only: wait for all of them (bounded)
  bool have = g < 0 || flag_load(P.fA + g) >= 1;
  for (uint32_t it = 0; !__all(have) && it < SPIN; it++) {
    __builtin_amdgcn_s_sleep(1);
    if (!have) have = flag_load(P.fA + g) >= 1;
  }
  have = have && g >= 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint64_t* r = P.recs + (have ? (uint64_t)g : 0) * R_WORDS;
  const uint32_t meta = have ? (uint32_t)st_load(r + R_META) : 0u;
  uint64_t ent[NENT / 2], out[NOUT][2];
#pragma unroll
  for (uint32_t q = 0; q < NENT / 2; q++) ent[q] = have ? st_load(r + R_ENT0 + q) : 0;
#pragma unroll
  for (uint32_t o = 0; o < NOUT; o++) {
    out[o][0] = have ? st_load(r + R_OUT0 + 2 * o) : 0;
    out[o][1] = have ? st_load(r + R_OUT0 + 2 * o + 1) : 0;
  }
  const uint32_t ne = meta & 0xFF, no = (meta >> 8) & 0xFF;
  L.bk_n[lane] = 0;
  wave_sync();
  // every outcome exit that lands inside a later window segment is a link candidate
#pragma unroll
  for (uint32_t o = 0; o < NOUT; o++) {
    if (o < no) {
      const uint64_t x = out[o][0];
      if (x < P.hi) {
        const int64_t u = (int64_t)(x / SEG) - w0;
        if (u > (int64_t)lane && u < (int64_t)WIN) {
          const uint32_t slot = atomicAdd(&L.bk_n[u], 1u);
          if (slot < BKT) L.bk[u][slot] = (uint32_t)(x - (uint64_t)(w0 + u) * SEG);
        }
      }
    }
  }
  if (lane == 0 && a >= -1 && !(E.st & S_PARTIAL)) {  // the exact anchor's exit supports too
    const int64_t u = (int64_t)(E.X / SEG) - w0;
    if (E.X < P.hi && u >= 0 && u < (int64_t)WIN) {
      const uint32_t slot = atomicAdd(&L.bk_n[u], 1u);
      if (slot < BKT) L.bk[u][slot] = (uint32_t)(E.X - (uint64_t)(w0 + u) * SEG);
    }
  }
  wave_sync();
  // each segment: the first entry that some exit lands on -> its outcome
  const uint32_t nb = L.bk_n[lane] < BKT ? L.bk_n[lane] : BKT;
  uint32_t oc = 0xFFu;
#pragma unroll
  for (uint32_t q = 0; q < NENT; q++) {
    const uint32_t e = (uint32_t)(ent[q / 2] >> (32 * (q % 2)));
    if (oc == 0xFFu && q < ne) {
      for (uint32_t b = 0; b < nb; b++)
        if (L.bk[lane][b] == (e & 0xFFFFu)) { oc = e >> 29; break; }
    }
  }
  uint64_t dX = 0, dW = 0;
#pragma unroll
  for (uint32_t o = 0; o < NOUT; o++)
    if (o == oc) { dX = out[o][0]; dW = out[o][1]; }
  // k's input: the trusted outcome of the nearest earlier segment that reaches k
  const uint64_t m = __ballot(oc != 0xFFu && lane < WIN - 1 && dX >= ts);
  cstate I;
  I.cnt = 0;
  if (!m) { I.X = 0; I.cov_ps = 0; I.cov_start = 0; I.cov_kw = 0; I.st = S_NONE; return I; }
  const uint32_t p = 63 - __builtin_clzll(m);
  const uint64_t pss = (uint64_t)(w0 + (int64_t)p) * SEG;
  const uint64_t w1 = rl64(dW, p);
  I.X = rl64(dX, p);
  I.cov_ps = pss + (w1 & 0xFFFFF);
  I.cov_start = I.cov_ps - ((w1 >> 20) & 0xF);
  I.cov_kw = (uint32_t)(w1 >> 32);
  I.st = 0;
  return I;
}

// Step C: is the assumed input of segment k exact? It is when some earlier
// segment a has an exact output and every segment j in (a, k] assumed exactly
// its predecessor's published output (pair flag fP[j] = 1); when a's exact
// output came from the slow path, segment a+1's input is compared with it
// directly. A decoupled look-back over 64 flags per round trip: pair flags are
// published from local work only, so nothing here waits on other validations.
XYWS_DEV bool validate_wave(const st_params& P, uint64_t k, uint32_t lane) {
  uint32_t* err = P.head + 1;
  for (int64_t b = (int64_t)k - 1, rounds = 0; rounds < 64; b -= 64, rounds++) {
    const int64_t j = b - (int64_t)lane;
    uint32_t fv = j >= 0 ? flag_load(P.fV + j) : (j == -1 ? 3u : 0u);
    const uint64_t mv = __ballot(fv >= 1);
    const uint32_t la = mv ? (uint32_t)__builtin_ctzll(mv) : 64u;
    // pair flags of the segments after the anchor (k's own pair is lane -1: checked by caller)
    uint32_t fp = (lane < la && j >= 0) ? flag_load(P.fP + j) : 1u;
    for (uint32_t it = 0; !__all(fp != 0) && it < SPIN; it++) {
      __builtin_amdgcn_s_sleep(1);
      if (fp == 0) fp = flag_load(P.fP + j);
    }
    if (!__all(fp != 0)) { atomicOr(err, 4u); return false; }
    if (__ballot(fp == 2)) return false;
    if (!mv) continue;  // all 64 pairs good, anchor further back
    const uint32_t fva = rl32(fv, la);
    if (fva == 2) {  // slow-path anchor: its successor must have assumed its exact output
      const int64_t a = b - (int64_t)la;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const cstate E = exact_out(P, a, 2);
      cstate In;
      if ((uint64_t)(a + 1) == k) return true;  // caller compares k's own input with it
      In = load_state(P.recs + (uint64_t)(a + 1) * R_WORDS + R_CI);
      return same_state(In, E);
    }
    return true;
  }
  return false;
}

// Step D: exclusive frame-count prefix of segment k (decoupled look-back sum).
XYWS_DEV uint64_t count_prefix(const st_params& P, uint64_t k, uint32_t lane) {
  uint32_t* err = P.head + 1;
  uint64_t sum = 0;
  int64_t b = (int64_t)k - 1;
  for (uint32_t guard = 0; b >= 0 && guard < (1u << 20); guard++) {
    const int64_t j = b - (int64_t)lane;
    uint32_t fn = j >= 0 ? flag_load(P.fN + j) : 2u;
    const uint64_t mi = __ballot(fn >= 2);
    const uint32_t li = mi ? (uint32_t)__builtin_ctzll(mi) : 64u;
    bool ready = lane >= li || fn >= 1;
    for (uint32_t it = 0; !__all(ready) && it < SPIN; it++) {
      __builtin_amdgcn_s_sleep(2);
      if (!ready) { fn = flag_load(P.fN + j); ready = fn >= 1; }
    }
    if (!__all(ready)) { atomicOr(err, 8u); return sum; }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint64_t v = 0;
    if (lane < li) v = st_load(P.recs + (uint64_t)j * R_WORDS + R_NA);
    else if (lane == li && j >= 0) v = st_load(P.recs + (uint64_t)j * R_WORDS + R_NI);
#pragma unroll
    for (uint32_t o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);  // lanes > li hold 0
    sum += v;
    if (mi) break;
    b -= 64;
  }
  return sum;
}

// The exact frames of segment k from input s (lane 0): the suffix of a primary
// walk of the survivor graph (mode 1), or an exact header chase (mode 2).
struct chain_res {
  cstate o;
  uint32_t mode, node, rem;  // mode 1: the path from survivor `node`, rem frames
};

XYWS_DEV chain_res own_chain(const st_params& P, st_lds& L, uint32_t nsurv, uint64_t ss,
                             uint64_t se, const cstate& s) {
  chain_res c;
  c.o = s; c.mode = 0; c.node = 0; c.rem = 0;
  if ((s.st & S_PARTIAL) || s.X >= se || s.X >= P.hi) return c;
  const uint32_t xr = (uint32_t)(s.X - ss);
  uint32_t x = 0, y = nsurv;
  while (x < y) {
    const uint32_t m = (x + y) >> 1;
    if (L.s_pos[m] < xr) x = m + 1; else y = m;
  }
  if (x < nsurv && L.s_pos[x] == xr && L.s_out[x] < NOUT) {
    const uint32_t oc = L.s_out[x];
    c.mode = 1;
    c.node = x;
    c.rem = L.s_rem[x];
    c.o.X = L.outs[oc][0]; c.o.cov_ps = L.outs[oc][1]; c.o.cov_start = L.outs[oc][2];
    c.o.cov_kw = (uint32_t)L.outs[oc][3];
    c.o.cnt = s.cnt + c.rem;
    c.o.st = 0;
  } else {
    c.mode = 2;
    bool inc = false;
    chase_global(P, c.o, se, 0xFFFFFFFFu, &inc);
  }
  return c;
}

// Block-wide exclusive scan of one value per thread (all threads call).
XYWS_DEV uint32_t block_scan(st_lds& L, uint32_t v, uint32_t lane, uint32_t wave, uint32_t& total) {
  uint32_t x = v;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  __syncthreads();
  if (lane == 63) L.scan[wave] = x;
  __syncthreads();
  uint32_t wb = 0, tot = 0;
#pragma unroll
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t si = L.scan[i];
    if (i < wave) wb += si;
    tot += si;
  }
  total = tot;
  return wb + x - v;
}

XYWS_DEV void write_frame(const st_params& P, uint64_t ord, uint64_t start, const hdr_info& h,
                          uint64_t ps, int32_t hdr_shift) {
  if (!P.frames || ord >= P.cap) return;
  xyws_frame f;
  f.frame_off = (int64_t)(start - P.lo) - hdr_shift;
  f.payload_off = (int64_t)(ps - P.lo);
  f.payload_len = h.plen;
  f.key[0] = (uint8_t)h.key; f.key[1] = (uint8_t)(h.key >> 8);
  f.key[2] = (uint8_t)(h.key >> 16); f.key[3] = (uint8_t)(h.key >> 24);
  f.flags = h.flags;
  f.hdr_len = (uint8_t)h.hlen;
  f.status = (uint8_t)(h.status | (sat_add(ps, h.plen) > P.hi ? XYWS_ST_PAYLOAD_INCOMPLETE : 0));
  f.reserved = 0;
  P.frames[ord] = f;
}

XYWS_DEV uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (uint32_t o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// XOR words for the 16-byte chunk at segment offset a. Entries are contiguous
// frames sorted by start; g = the last entry starting at or before a. Common
// case: one frame's payload covers the whole chunk.
XYWS_DEV u32x4 chunk_xor(const st_lds& L, uint32_t nfl, uint32_t g, uint32_t a) {
  const fent e = L.flist[g];
  if (e.ps <= a && e.end >= a + 16) return u32x4{e.kw, e.kw, e.kw, e.kw};
  u32x4 w = {0u, 0u, 0u, 0u};
  for (uint32_t h = g; h < nfl; h++) {
    const fent f = L.flist[h];
    if (h != g && f.start >= a + 16) break;
    w.x |= f.kw & range_mask(a, f.ps, f.end);
    w.y |= f.kw & range_mask(a + 4, f.ps, f.end);
    w.z |= f.kw & range_mask(a + 8, f.ps, f.end);
    w.w |= f.kw & range_mask(a + 12, f.ps, f.end);
  }
  return w;
}

// ---------------------------------------------------------------- kernel
__global__ void __launch_bounds__(NT, 2) k_stream_fused(st_params P) {
  __shared__ st_lds L;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint32_t* err = P.head + 1;
  const bool want_unmasked = (P.opts & XYWS_OPT_UNMASKED_HINT) != 0;
  const bool parse_only = (P.opts & XYWS_OPT_PARSE_ONLY) != 0;
  const uint64_t lo = P.lo, hi = P.hi;

  for (;;) {
    if (tid == 0) L.seg_id = atomicAdd(P.head, 1u);
    __syncthreads();
    const uint64_t seg = L.seg_id;
    if (seg >= P.nseg) break;
    uint64_t tstamp = stat_on(P) ? __builtin_amdgcn_s_memtime() : 0;
    const uint64_t ss = seg * SEG, se = ss + SEG;

    // ---- 1. loads: the whole segment into registers -----------------------
    // Buffer descriptor over [ss, ss + round16(hi - ss)) capped at SEG + 16:
    // the base and range live in SGPRs, each lane keeps one 32-bit offset, and
    // chunks past the batch read as zero (hardware range check).
    const uint64_t room = hi - ss;
    const uint32_t nrec = room >= SEG + 16 ? SEG + 16 : (uint32_t)((room + 15) & ~15ull);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(P.base + ss, 0, nrec, 0x00020000);
    const uint32_t voff = tid * 16u;
    u32x4 d[CHS];
#pragma unroll
    for (uint32_t k = 0; k < CHS; k++) d[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, k * NT * 16u, 0);
    u32x4 halo = {0u, 0u, 0u, 0u};
    if (tid == 0) halo = __builtin_amdgcn_raw_buffer_load_b128(rs, 0, SEG, 0);
    if (tid == 0) { L.nsurv = 0; L.overflow = 0; }

    // ---- 1b. per sub-tile: LDS copy, prefilter, candidates -> survivors ----
#pragma nounroll
    for (uint32_t s = 0; s < NSUB; s++) {
      const uint64_t ts = ss + (uint64_t)s * SUB, te = ts + SUB;
      __syncthreads();  // previous sub-tile fully consumed
#pragma unroll
      for (uint32_t k = 0; k < CHSUB; k++) {
        const u32x4 v = s == 0 ? d[k] : d[CHSUB + k];
        *reinterpret_cast<u32x4*>(&L.sub[(k * NT + tid) * 16u]) = v;
      }
      if (tid == 0) {
        const u32x4 v = s == 0 ? d[CHSUB] : halo;
        *reinterpret_cast<u32x4*>(&L.sub[SUB]) = v;
      }
      __syncthreads();
      // prefilter: lane owns sub-tile positions [tid*128, tid*128+128)
      uint64_t cand[2] = {0, 0};
      {
        const uint32_t p0 = tid * 128u;
        uint32_t w = *reinterpret_cast<const uint32_t*>(&L.sub[p0]);
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) {
          const uint32_t wn = *reinterpret_cast<const uint32_t*>(&L.sub[p0 + 4 * i + 4]);
          const uint32_t b1s = (w >> 8) | (wn << 24);  // byte t = byte at position 4i+t+1
          const uint32_t rsv_ok = ~((w & 0x70707070u) + 0x70707070u) & 0x80808080u;
          const uint32_t bad_op = ((w << 5) | ((w & (w >> 1)) << 7)) & 0x80808080u;
          const uint32_t m_ok = (want_unmasked ? ~b1s : b1s) & 0x80808080u;
          const uint32_t c = rsv_ok & ~bad_op & m_ok;
          const uint32_t nib = ((c >> 7) | (c >> 14) | (c >> 21) | (c >> 28)) & 0xFu;
          cand[i >> 4] |= (uint64_t)nib << (4 * (i & 15));
          w = wn;
        }
        const uint64_t a0 = ts + p0;
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
          const uint64_t st = a0 + 64 * h;
          uint64_t m = ~0ull;
          if (st + 64 > hi) m = (st >= hi) ? 0 : ((1ull << (hi - st)) - 1);
          if (st < lo) m &= (lo - st >= 64) ? 0 : ~((1ull << (lo - st)) - 1);
          cand[h] &= m;
          L.bits[2 * tid + h] = cand[h];
        }
      }
      __syncthreads();
      // full parse of the lane's candidates
      uint64_t surv[2] = {0, 0};
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        uint64_t m = cand[h];
        while (m) {
          const uint32_t b = __builtin_ctzll(m);
          m &= m - 1;
          const uint32_t prel = tid * 128u + 64u * h + b;
          const uint64_t pabs = ts + prel;
          hdr_info hh = header_lds(L.sub, prel, pabs, hi);
          if (!plausible(hh, L.sub[prel + 1])) continue;
          const uint64_t nx = sat_add(pabs + hh.hlen, hh.plen);
          if (nx > hi) continue;
          bool ok = true;
          if (nx < te) {
            const uint32_t nr = (uint32_t)(nx - ts);
            ok = (L.bits[nr >> 6] >> (nr & 63)) & 1ull;
          }
          if (ok) surv[h] |= 1ull << b;
        }
      }
      // ordered append: block-exclusive scan of per-lane survivor counts
      const uint32_t c0 = __popcll(surv[0]), c1 = __popcll(surv[1]);
      const uint32_t v = c0 + c1;
      uint32_t x = v;
#pragma unroll
      for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (lane == 63) L.scan[wave] = x;
      __syncthreads();
      uint32_t wb = 0, tot = 0;
#pragma unroll
      for (uint32_t i = 0; i < 4; i++) {
        const uint32_t si = L.scan[i];
        if (i < wave) wb += si;
        tot += si;
      }
      const uint32_t base_n = L.nsurv;
      const bool fits = base_n + tot <= SMAX;
      if (fits) {
        uint32_t r = base_n + wb + x - v;
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
          uint64_t m = surv[h];
          while (m) {
            const uint32_t b = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t prel = tid * 128u + 64u * h + b;
            hdr_info hh = header_lds(L.sub, prel, ts + prel, hi);
            L.s_pos[r] = s * SUB + prel;
            L.s_nrel[r] = clamp_rel(sat_add(ts + prel + hh.hlen, hh.plen), ss);
            L.s_key[r] = hh.key;
            L.s_hlen[r] = (uint8_t)hh.hlen;
            r++;
          }
        }
      }
      __syncthreads();
      if (tid == 0) {
        if (fits) L.nsurv = base_n + tot;
        else L.overflow = 1;
      }
    }
    __syncthreads();

    // ---- 2. link survivors ------------------------------------------------
    const uint32_t nsurv = L.overflow ? 0u : L.nsurv;
    for (uint32_t i = tid; i < nsurv; i += NT) {
      const uint32_t nr = L.s_nrel[i];
      uint16_t nn = N_EXIT;
      if (nr < SEG) {
        uint32_t x = i + 1, y = nsurv;  // successor lies after i: search (i, nsurv)
        while (x < y) {
          const uint32_t m = (x + y) >> 1;
          if (L.s_pos[m] < nr) x = m + 1; else y = m;
        }
        nn = (x < nsurv && L.s_pos[x] == nr) ? (uint16_t)x : N_DEAD;
      }
      L.s_nxt[i] = nn;
      L.s_jmp[0][i] = (nn == N_EXIT || nn == N_DEAD) ? J_TERM : nn;
      L.s_rem[i] = 1;
      L.s_last[i] = nn == N_EXIT ? (uint16_t)i : (nn == N_DEAD ? T_DEAD : 0);
    }
    __syncthreads();

    // ---- 2a. pointer doubling over the survivor graph (all threads) --------
    // After round b, s_jmp[b][i] is the 2^b-th successor of i; s_rem and
    // s_last converge to the frames to the chain end and its last node.
    for (uint32_t b = 0; b + 1 < LV; b++) {
      uint32_t nj[2], nr[2], nl[2];
      bool any = false;
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t i = tid + h * NT;
        nj[h] = J_TERM; nr[h] = 0; nl[h] = 0;
        if (i < nsurv) {
          const uint32_t j = L.s_jmp[b][i];
          nr[h] = L.s_rem[i];
          nl[h] = L.s_last[i];
          if (j != J_TERM) {
            const uint32_t jj = L.s_jmp[b][j];
            nj[h] = jj;
            nr[h] += L.s_rem[j];
            if (jj == J_TERM) nl[h] = L.s_last[j];
            any = true;
          }
        }
      }
      const bool more = __syncthreads_or(any);
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t i = tid + h * NT;
        if (i < nsurv) {
          L.s_jmp[b + 1][i] = (uint16_t)nj[h];
          L.s_rem[i] = (uint16_t)nr[h];
          L.s_last[i] = (uint16_t)nl[h];
        }
      }
      __syncthreads();
      if (!more) {  // every chain resolved: the remaining levels are all J_TERM
        for (uint32_t bb = b + 2; bb < LV; bb++)
          for (uint32_t i = tid; i < nsurv; i += NT) L.s_jmp[bb][i] = J_TERM;
        break;
      }
    }
    // outcome ids: chain-end nodes ranked in position order
    {
      uint32_t isl[2];
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t i = 2 * tid + h;
        isl[h] = (i < nsurv && L.s_nxt[i] == N_EXIT) ? 1u : 0u;
      }
      uint32_t tot;
      const uint32_t r0 = block_scan(L, isl[0] + isl[1], lane, wave, tot);
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t i = 2 * tid + h;
        if (isl[h]) {
          const uint32_t id = r0 + (h ? isl[0] : 0);
          L.s_out[i] = id < NOUT ? (uint8_t)id : O_UNREC;
          if (id < NOUT) {
            const uint64_t pp = ss + L.s_pos[i];
            const uint64_t ps = pp + L.s_hlen[i];
            L.outs[id][0] = L.s_nrel[i] == 0xFFFFFFFFu ? ~0ull : ss + L.s_nrel[i];
            L.outs[id][1] = ps;
            L.outs[id][2] = pp;
            L.outs[id][3] = aligned_key(L.s_key[i], ps, 0);
          }
        }
      }
      if (tid == 0) L.nout_pub = tot < NOUT ? tot : NOUT;
      __syncthreads();
      // every node's outcome = its chain end's; entries = the first NENT exiting nodes
      uint32_t ex[2];
      uint8_t oc[2];
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t i = 2 * tid + h;
        oc[h] = O_DEAD;
        if (i < nsurv) {
          const uint32_t t = L.s_last[i];
          oc[h] = t == T_DEAD ? O_DEAD : L.s_out[t];
        }
        ex[h] = oc[h] < NOUT ? 1u : 0u;
      }
      __syncthreads();
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t i = 2 * tid + h;
        if (i < nsurv) L.s_out[i] = oc[h];
      }
      const uint32_t e0 = block_scan(L, ex[0] + ex[1], lane, wave, tot);
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t i = 2 * tid + h;
        const uint32_t q = e0 + (h ? ex[0] : 0);
        if (ex[h] && q < NENT) L.ents[q] = L.s_pos[i] | ((uint32_t)L.s_rem[i] << 16) | ((uint32_t)oc[h] << 29);
      }
      if (tid == 0) L.nent_pub = tot < NENT ? tot : NENT;
    }
    __syncthreads();

    // ---- 2b/3/4/5a: wave 0: graph walk + aggregate (lane 0), look-back
    //      (wave), own resolution (lane 0), helping (wave) ------------------------
    if (wid0(wave)) stat_phase(P, ST_T_PASS1, tstamp);
    if (wave == 0) {
      {  // publish the aggregate: lanes store words in parallel, one drain, one flag
        uint64_t* rec = P.recs + seg * R_WORDS;
        const uint32_t nent = L.nent_pub, nout = L.nout_pub;
        if (lane == 0)
          st_store(rec + R_META, (uint64_t)nent | ((uint64_t)nout << 8) | ((uint64_t)L.overflow << 16));
        if (lane < (nent + 1) / 2) {
          const uint32_t q = 2 * lane;
          st_store(rec + R_ENT0 + lane, (uint64_t)L.ents[q] | (q + 1 < nent ? (uint64_t)L.ents[q + 1] << 32 : 0));
        }
        if (lane >= 16 && lane < 16 + nout) {
          const uint32_t o = lane - 16;
          st_store(rec + R_OUT0 + 2 * o, L.outs[o][0]);
          st_store(rec + R_OUT0 + 2 * o + 1, (L.outs[o][1] - ss) | ((L.outs[o][1] - L.outs[o][2]) << 20) |
                                                 (L.outs[o][3] << 32));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(P.fA + seg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }

      stat_phase(P, ST_T_WALK, tstamp);
      // ---- 4. input state: exact, or speculated from the aggregates (wave)
      bool exact = false;
      cstate I = resolve_input(P, L, seg, lane, exact);
      stat_phase(P, ST_T_INPUT, tstamp);
      const bool spec = !exact && !(I.st & S_NONE);
      uint64_t* rec = P.recs + seg * R_WORDS;

      // ---- 5a. own frames from that input (lane 0); publish (input, output)
      chain_res c;
      if (lane == 0) {
        if (exact || spec) {
          c = own_chain(P, L, nsurv, ss, se, I);
          store_state(rec + R_CI, I);
          store_state(rec + R_CO, c.o);
          st_store(rec + R_CN, c.o.cnt);
          flag_publish(P.fC + seg, 1u);
          if (exact) flag_publish(P.fV + seg, 1u);
        } else {
          c.mode = 0;  // placeholder: resolved by the slow path below
        }
      }
      if (stat_on(P)) stat_add(P, exact ? ST_EXACT_IN : spec ? ST_SPEC : ST_NOSPEC, 1);
      stat_phase(P, ST_T_CHAIN, tstamp);

      // ---- 5b. own pair flag: assumed input == predecessor's published output
      bool ok = exact;
      if (spec) {
        uint32_t fc = 0;
        for (uint32_t it = 0; it < SPIN; it++) {
          fc = flag_load(P.fC + seg - 1);
          if (fc >= 1) break;
          __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const cstate Op = load_state(P.recs + (seg - 1) * R_WORDS + R_CO);
        const bool pair = fc >= 1 && same_state(I, Op);
        if (lane == 0) flag_publish(P.fP + seg, pair ? 1u : 2u);
        // ---- 5c. validation (wave): pair flags back to an exact segment
        if (pair) {
          ok = validate_wave(P, seg, lane);
          if (ok) {  // a slow-path predecessor anchor: compare with its exact output
            const uint32_t fvp = flag_load(P.fV + seg - 1);
            if (fvp == 2) ok = same_state(I, exact_out(P, (int64_t)seg - 1, 2));
          }
        }
      } else if (lane == 0) {
        flag_publish(P.fP + seg, exact ? 1u : 2u);
      }
      // otherwise wait for the predecessor's exact output (slow path)
      if (!ok) {
        if (stat_on(P)) stat_add(P, ST_SLOW, 1);
        uint32_t fvp = 0;
        for (uint32_t it = 0; it < SPIN; it++) {
          fvp = flag_load(P.fV + seg - 1);
          if (fvp >= 1) break;
          __builtin_amdgcn_s_sleep(2);
        }
        if (fvp == 0) atomicOr(P.head + 1, 16u);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        cstate E = exact_out(P, (int64_t)seg - 1, fvp);
        E.cnt = 0;
        if (spec && same_state(E, I)) {
          ok = true;  // the speculation was right after all
          if (lane == 0) flag_publish(P.fV + seg, 1u);
        } else {
          if (stat_on(P)) stat_add(P, ST_RECOMP, 1);
          I = E;
          if (lane == 0) {
            c = own_chain(P, L, nsurv, ss, se, I);
            if (!spec) {  // nothing published yet: the exact pair serves the validators
              store_state(rec + R_CI, I);
              store_state(rec + R_CO, c.o);
              st_store(rec + R_CN, c.o.cnt);
              flag_publish(P.fC + seg, 1u);
            }
            store_state(rec + R_EX, c.o);
            st_store(rec + R_EN, c.o.cnt);
            flag_publish(P.fV + seg, 2u);
          }
        }
      } else if (spec && lane == 0) {
        flag_publish(P.fV + seg, 1u);
      }
      if (stat_on(P) && ok && spec) stat_add(P, ST_VALID, 1);
      stat_phase(P, ST_T_VALID, tstamp);

      // ---- 5c. frame count: aggregate + prefix (only ordinals need it) ------
      uint64_t n = rl64(lane == 0 ? c.o.cnt : 0, 0);
      if (lane == 0) {
        st_store(rec + R_NA, n);
        flag_publish(P.fN + seg, 1u);
        atomicAdd(reinterpret_cast<unsigned long long*>(P.head + 4), (unsigned long long)n);
      }
      uint64_t nbase = 0;
      if (P.frames) {
        nbase = count_prefix(P, seg, lane);
        if (lane == 0) {
          st_store(rec + R_NI, nbase + n);
          flag_publish(P.fN + seg, 2u);
        }
      }
      if (lane == 0) {
        L.in = I;
        L.out = c.o;
        L.mode = c.mode;
        L.node_x = c.node;
        L.rem_x = c.rem;
        L.nbase = nbase;
        stat_phase(P, ST_T_COUNT, tstamp);
        if (stat_on(P)) {
          stat_add(P, c.mode == 2 ? ST_MODE2 : ST_MODE1, 1);
          stat_add(P, ST_NSURV, nsurv);
        }
      }
    }
    __syncthreads();

    // ---- 5b/6. frame-list passes, XOR into registers -------------------------
    const cstate sin = L.in;
    const uint32_t mode = L.mode;
    const uint64_t fb = L.nbase + sin.cnt;  // ordinal of the first frame starting in this segment
    uint32_t changed = 0;

    // the carried-header frame of the batch is described by segment 0
    if (seg == 0 && tid == 0 && (sin.st & S_HDRCARRY) && !(sin.st & S_PARTIAL)) {
      hdr_info hh = header_carried(P.base, lo, hi, P.cin);
      write_frame(P, 0, lo, hh, sin.cov_ps, (int32_t)P.cin->hdr_len);
    }
    if (tid == 0) {
      L.nfl = 0;
      if (!(sin.st & (S_NOCOV | S_PARTCARRY))) {  // covering entry: frame begun before ss
        fent e;
        e.start = 0;
        e.ps = clamp_rel(sin.cov_ps, ss);
        e.end = clamp_rel(sin.X, ss);
        e.kw = sin.cov_kw;
        L.flist[0] = e;
        L.nfl = 1;
      }
      L.fbase = fb;
      L.chase_X = sin.X;
      L.pass_done = (mode != 2);
    }
    __syncthreads();
    if (mode == 1) {
      // frame d of the path from node x is its d-th successor: binary lifting
      const uint32_t x0 = L.node_x, rem = L.rem_x, base_n = L.nfl;
      for (uint32_t dd = tid; dd < rem && base_n + dd < FCAP; dd += NT) {
        uint32_t i = x0;
#pragma unroll
        for (uint32_t bb = 0; bb < LV; bb++)
          if ((dd >> bb) & 1u) i = L.s_jmp[bb][i];
        const uint64_t p = ss + L.s_pos[i];
        const uint64_t ps = p + L.s_hlen[i];
        fent e;
        e.start = L.s_pos[i];
        e.ps = (uint32_t)(ps - ss);
        e.end = L.s_nrel[i];
        e.kw = aligned_key(L.s_key[i], ps, 0);
        L.flist[base_n + dd] = e;
        if (P.frames) {
          hdr_info hh = header_global(P.base, p, hi);
          write_frame(P, fb + dd, p, hh, ps, 0);
        }
      }
      __syncthreads();
      if (tid == 0) L.nfl = base_n + rem;
    }

    for (;;) {
      if (mode == 2 && tid == 0) {  // exact chase in global memory, FCAP entries per pass
        uint64_t X = L.chase_X, ord = L.fbase;
        uint32_t n = L.nfl;
        const uint64_t stop = se < hi ? se : hi;
        while (X < stop && n < FCAP) {
          hdr_info hh = header_global(P.base, X, hi);
          if (!hh.hlen) { X = ~0ull; break; }
          const uint64_t ps = X + hh.hlen;
          fent e;
          e.start = (uint32_t)(X - ss);
          e.ps = (uint32_t)(ps - ss);
          e.end = clamp_rel(sat_add(ps, hh.plen), ss);
          e.kw = aligned_key(hh.key, ps, 0);
          L.flist[n++] = e;
          write_frame(P, ord++, X, hh, ps, 0);
          X = sat_add(ps, hh.plen);
        }
        L.nfl = n;
        L.fbase = ord;
        L.chase_X = X;
        L.pass_done = !(X < stop);
      }
      __syncthreads();
      const uint32_t nfl = L.nfl;
      if (!parse_only && nfl) {
        uint32_t g = 0;
#pragma unroll
        for (uint32_t k = 0; k < CHS; k++) {
          const uint32_t a = (k * NT + tid) * 16u;  // increases with k: g only moves forward
          while (g + 1 < nfl && L.flist[g + 1].start <= a) g++;
          const u32x4 x = chunk_xor(L, nfl, g, a);
          if ((x.x | x.y | x.z | x.w) != 0u) {
            d[k] ^= x;
            changed |= 1u << k;
          }
        }
      }
      const uint32_t done = L.pass_done;
      __syncthreads();
      if (done) break;
      if (tid == 0) {  // next pass: the last frame becomes the covering entry
        fent e = L.flist[L.nfl - 1];
        e.start = 0;
        L.flist[0] = e;
        L.nfl = 1;
      }
      __syncthreads();
    }

    if (wid0(wave)) stat_phase(P, ST_T_XOR, tstamp);
    // ---- 6b. store changed chunks ------------------------------------------
    if (!parse_only) {
#pragma unroll
      for (uint32_t k = 0; k < CHS; k++) {
        if (!((changed >> k) & 1u)) continue;
        const uint64_t a = ss + (k * NT + tid) * 16u;
        if (a >= lo && a + 16 <= hi) {
          __builtin_amdgcn_raw_buffer_store_b128(d[k], rs, voff, k * NT * 16u, 0);
        } else {  // edge chunk: only the caller's bytes, only changed ones
          const uint32_t w[4] = {d[k].x, d[k].y, d[k].z, d[k].w};
          for (uint32_t t = 0; t < 16; t++) {
            const uint64_t q = a + t;
            const uint8_t nb = (uint8_t)(w[t >> 2] >> (8u * (t & 3u)));
            if (q >= lo && q < hi && P.base[q] != nb) P.base[q] = nb;
          }
        }
      }
    }

    if (wid0(wave)) stat_phase(P, ST_T_STORE, tstamp);
    // ---- the last workgroup to finish: frame count + carry out -------------
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const uint32_t done = atomicAdd(P.head + 2, 1u);
      if (done == P.nseg - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const uint64_t total = __hip_atomic_load(reinterpret_cast<uint64_t*>(P.head + 4),
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t fvl = flag_load(P.fV + P.nseg - 1);
        const cstate o = exact_out(P, (int64_t)P.nseg - 1, fvl);
        if (P.nframes) *P.nframes = total;
        if (P.cout) {
          xyws_carry c;
          for (int i = 0; i < 64; i++) reinterpret_cast<uint8_t*>(&c)[i] = 0;
          c.frames_total = P.cin->frames_total + total;
          if (o.st & S_PARTIAL) {
            uint32_t nb = 0;
            if (o.st & S_PARTCARRY) {
              for (; nb < P.cin->hdr_len; nb++) c.hdr[nb] = P.cin->hdr[nb];
              for (uint64_t q = lo; q < hi && nb < 14; q++) c.hdr[nb++] = P.base[q];
            } else {
              for (uint64_t q = o.X; q < hi && nb < 14; q++) c.hdr[nb++] = P.base[q];
            }
            c.hdr_len = (uint8_t)nb;
          } else if (o.X > hi && !(o.st & S_NOCOV)) {
            if (o.st & S_CARRIED) {
              c.payload_remaining = P.cin->payload_remaining - (hi - lo);
              c.phase = P.cin->phase + (hi - lo);
              for (int i = 0; i < 4; i++) c.key[i] = P.cin->key[i];
            } else {
              const hdr_info hh = (o.st & S_HDRCARRY) ? header_carried(P.base, lo, hi, P.cin)
                                                      : header_global(P.base, o.cov_start, hi);
              c.payload_remaining = hh.plen - (hi - o.cov_ps);
              c.phase = hi - o.cov_ps;
              c.key[0] = (uint8_t)hh.key; c.key[1] = (uint8_t)(hh.key >> 8);
              c.key[2] = (uint8_t)(hh.key >> 16); c.key[3] = (uint8_t)(hh.key >> 24);
            }
          }
          *P.cout = c;
        }
      }
    }
    __syncthreads();
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

constexpr uint64_t HEAD_BYTES = 512;  // [0] ticket, [1] error, [64..128) carry snapshot, [128..384) stats

int occupancy_grid() {
  static int cached = 0;
  if (cached) return cached;
  int dev = 0, cus = 256, per = 2;
  (void)hipGetDevice(&dev);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_stream_fused, NT, 0) != hipSuccess || per < 1)
    per = 2;
  cached = cus * per;
  return cached;
}

}  // namespace

void stream_scratch_init(stream_scratch* s) {
  s->mem = nullptr;
  s->bytes = 0;
  s->max_tiles = 0;
}

void stream_scratch_free(stream_scratch* s) {
  if (s->mem) (void)hipFree(s->mem);
  s->mem = nullptr;
  s->bytes = 0;
  s->max_tiles = 0;
}

static uint64_t flags_bytes(uint64_t n) { return (5 * n * 4 + 255) & ~255ull; }  // fA fC fV fN fP

static int scratch_grow(stream_scratch* s, uint64_t segs) {
  if (s->mem && segs <= s->max_tiles) return XYWS_OK;
  const uint64_t want = segs < 64 ? 64 : segs;
  const uint64_t bytes = HEAD_BYTES + flags_bytes(want) + want * R_WORDS * 8;
  void* m = nullptr;
  if (hipMalloc(&m, bytes) != hipSuccess) return XYWS_ERR_NOMEM;
  if (s->mem) {
    (void)hipDeviceSynchronize();
    (void)hipFree(s->mem);
  }
  s->mem = m;
  s->bytes = bytes;
  s->max_tiles = want;
  return hipMemset(m, 0, HEAD_BYTES) == hipSuccess ? XYWS_OK : XYWS_ERR_HIP;
}

int stream_scratch_reserve(stream_scratch* s, uint64_t max_batch_bytes) {
  return scratch_grow(s, (max_batch_bytes + 15 + SEG - 1) / SEG + 1);
}

int stream_scratch_stats(stream_scratch* s, uint64_t out[32]) {
  if (!s->mem) return XYWS_ERR_INVALID;
  if (hipDeviceSynchronize() != hipSuccess) return XYWS_ERR_HIP;
  return hipMemcpy(out, static_cast<uint8_t*>(s->mem) + 128, 256, hipMemcpyDeviceToHost) == hipSuccess
             ? XYWS_OK : XYWS_ERR_HIP;
}

uint32_t stream_scratch_error(stream_scratch* s) {
  if (!s->mem) return 0;
  uint32_t v[2] = {0, 0};
  if (hipMemcpy(v, s->mem, 8, hipMemcpyDeviceToHost) != hipSuccess) return 0xFFFFFFFFu;
  return v[1];
}

int stream_decode_fused(stream_scratch* s, uint8_t* base, uint64_t lo, uint64_t hi,
                        const xyws_carry* cin, xyws_carry* cout, xyws_frame* frames, uint64_t cap,
                        uint64_t* nframes, uint32_t opts, hipStream_t stream) {
  if (hi == lo) {
    hipLaunchKernelGGL(k_stream_empty, dim3(1), dim3(64), 0, stream, cin, cout, nframes);
    return hipGetLastError() == hipSuccess ? XYWS_OK : XYWS_ERR_HIP;
  }
  const uint64_t nseg = (hi + SEG - 1) / SEG;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(stream, &cs);
  if (nseg > s->max_tiles || !s->mem) {
    if (cs != hipStreamCaptureStatusNone) return XYWS_ERR_CAPACITY;
    const int rc = scratch_grow(s, nseg);
    if (rc) return rc;
  }
  uint8_t* m = static_cast<uint8_t*>(s->mem);
  st_params P;
  P.base = base; P.lo = lo; P.hi = hi; P.nseg = nseg;
  P.cout = cout; P.frames = frames; P.cap = cap; P.nframes = nframes;
  P.head = reinterpret_cast<uint32_t*>(m);
  uint32_t* fl = reinterpret_cast<uint32_t*>(m + HEAD_BYTES);
  P.fA = fl;
  P.fC = fl + nseg;
  P.fV = fl + 2 * nseg;
  P.fN = fl + 3 * nseg;
  P.fP = fl + 4 * nseg;
  P.recs = reinterpret_cast<uint64_t*>(m + HEAD_BYTES + flags_bytes(s->max_tiles));
  P.opts = opts;
  // Ticket + flags zeroed every call (the error word [1] is sticky until read
  // back). The carry is snapshotted first: dev_carry_in may alias
  // dev_carry_out, which the last segment writes while others may still read
  // the incoming carry.
  xyws_carry* snap = reinterpret_cast<xyws_carry*>(m + 64);
  if (hipMemsetAsync(P.head + 2, 0, 24, stream) != hipSuccess) return XYWS_ERR_HIP;  // done, total
  if (hipMemsetAsync(P.head, 0, 4, stream) != hipSuccess) return XYWS_ERR_HIP;
  if ((opts & XYWS_OPT_STATS) && hipMemsetAsync(m + 128, 0, 256, stream) != hipSuccess) return XYWS_ERR_HIP;
  if (cin) {
    if (hipMemcpyAsync(snap, cin, sizeof(xyws_carry), hipMemcpyDeviceToDevice, stream) != hipSuccess)
      return XYWS_ERR_HIP;
  } else if (hipMemsetAsync(snap, 0, sizeof(xyws_carry), stream) != hipSuccess) {
    return XYWS_ERR_HIP;
  }
  P.cin = snap;
  if (hipMemsetAsync(fl, 0, (5 * nseg * 4 + 15) & ~15ull, stream) != hipSuccess) return XYWS_ERR_HIP;
  int grid = occupancy_grid();
  if ((uint64_t)grid > nseg) grid = (int)nseg;
  hipLaunchKernelGGL(k_stream_fused, dim3(grid), dim3(NT), 0, stream, P);
  return hipGetLastError() == hipSuccess ? XYWS_OK : XYWS_ERR_HIP;
}
