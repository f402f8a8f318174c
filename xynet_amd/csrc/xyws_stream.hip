// xyws_stream.hip — fused stream decoder for gfx950 (default mode of
// xyws_decode_stream).
//
// Problem: in a back-to-back batch the start of frame k+1 is known only after
// the header of frame k is parsed (websocket_frame_header.h:305-385 gives the
// header size and the payload length), so frame boundaries form a linked list
// through the batch. A serial chase from HBM costs one dependent load per
// frame, far below the HBM roofline.
//
// Geometry: a SEGMENT is 64 KiB; a persistent 512-thread workgroup takes
// segments by atomic ticket and runs a two-stage software pipeline over them:
// in each iteration it INDEXES its new segment t and then UNMASKS the segment
// it indexed in the previous iteration. The lag of one index phase is what
// lets the unmask stage run without waiting: by then every aggregate the
// speculation needs has long been published.
//
// INDEX(t) — local work only, never waits:
//  1. Load the segment (16 chunks of 16 B per lane, buffer descriptor with
//     base and range in SGPRs). For each 16 KiB sub-tile: stage it (+16 B
//     halo) in LDS, SWAR-prefilter every byte position for a plausible client
//     header (RSV = 0, known opcode, MASK as expected), check each candidate's
//     successor (position + header + length) is itself a candidate, and append
//     the survivors in position order.
//  2. Link survivors (successor = survivor at pos + H + len, EXIT past the
//     segment, DEAD otherwise); pointer doubling gives every node its 2^b-th
//     successors, its frame count to the chain end and its chain end.
//  3. Publish the AGGREGATE record: the first 16 nodes whose chain leaves the
//     segment (position, outcome, count), up to 8 outcomes (exit, last frame),
//     and the first 32 bytes of the segment (headers straddling into it are
//     read from this copy: the bytes themselves may be unmasked meanwhile).
// UNMASK(k):
//  4. Input state by speculation over the aggregates of the 63 preceding
//     segments: an entry node is trusted when some outcome of an earlier
//     segment (or the batch start) exits exactly onto it ("link support"); k
//     takes the trusted outcome of the nearest segment that reaches it.
//     Without one, it takes the nearest published output that reaches it.
//  5. Own frames from that input: the path from the entry survivor through
//     the jump tables (binary lifting, one frame per thread), or an exact
//     header chase. Publish (assumed input, output); the second of segments
//     k-1 and k to publish compares k's input with k-1's output ("pair").
//  6. XOR words for every chunk from the frame list, then load, XOR, store
//     the chunks that change (one read and one write of the payload; the
//     re-read of the lagged segment is served by the Infinity Cache).
// Validation is deferred: segment 0's input is exact, so when every pair
// matches, every input is exact by induction. The last workgroup to exit
// checks that; on a mismatch it repairs in order from the first bad pair:
// undo the wrong frames (XOR is an involution; a wrong chain never XORs its
// own header bytes, so it is re-derived from the bytes as they stand), redo
// with the exact input, until inputs match again. Speculation decides speed
// only; any byte stream (RSV bits, reserved opcodes, unmasked or non-minimal
// frames) decodes exactly as the reference parses it.
//
// Inter-workgroup hand-off follows MI355X_MICROARCH.md §Workgroup dispatch:
// record words are written with agent-scope (sc1) stores, drained with
// s_waitcnt vmcnt(0), then an sc1 flag store or agent-scope atomic; readers
// poll with sc1 loads. Flags and counters are zeroed by hipMemsetAsync before
// every launch. Every spin is bounded and reports through the device error
// word. Deadlock freedom: every wait points to a segment whose ticket was
// taken earlier (or to k+1, whose ticket was taken before this workgroup's
// current one), and the holder of such a ticket runs its index phase before
// anything that can wait.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xyws_stream.h"
#include "xyws_device.h"

namespace {

constexpr uint32_t SEG = 65536;            // segment bytes
constexpr uint32_t SUB = 8192;             // sub-tile bytes staged in LDS
constexpr uint32_t NSUB = SEG / SUB;       // 8
constexpr uint32_t NT = 256;               // threads per workgroup (4 waves)
constexpr uint32_t NW = NT / 64;           // waves per workgroup
constexpr uint32_t CHS = SEG / (16 * NT);  // 16 chunks of 16 B per lane
constexpr uint32_t CHSUB = SUB / (16 * NT);  // 2 per sub-tile
constexpr uint32_t PPL = SUB / NT;         // prefilter positions per lane (32)
constexpr uint32_t HALO = 16;
constexpr uint32_t SMAX = 512;             // survivors tracked per segment
constexpr uint32_t LV = 9;                 // jump-table levels: 2^LV >= SMAX
constexpr uint32_t NPT = SMAX / NT;        // survivor nodes per thread (2)
constexpr uint32_t FCAP = SUB / 16;        // frame-list entries per pass (overlays the sub-tile)
constexpr uint32_t NENT = 16;              // aggregate entry nodes (2 per record word)
constexpr uint32_t NOUT = 8;               // aggregate outcomes (2 record words each)
constexpr uint32_t SPIN = 1u << 24;        // bounded spins (~1 s)
constexpr uint32_t WIN = 64;               // segments seen by one speculation (one per lane)
constexpr uint32_t BKT = 8;                // exits kept per target segment during speculation
constexpr uint32_t OOB = 0x80000000u;      // buffer offset past every range: load 0, store dropped

constexpr uint16_t N_EXIT = 0xFFFF, N_DEAD = 0xFFFE;
constexpr uint8_t O_DEAD = 0xFE, O_UNREC = 0xFD;  // node outcome marks
constexpr uint16_t J_TERM = 0xFFFF;        // jump past the end of a chain
constexpr uint16_t T_DEAD = 0xFFFF;        // chain ends in a dead end

// composition-state bits
constexpr uint32_t S_PARTIAL = 1;    // stream ended in an incomplete header at X
constexpr uint32_t S_NOCOV = 2;      // no frame covers the bytes before X
constexpr uint32_t S_CARRIED = 4;    // covering frame = the open frame carried in
constexpr uint32_t S_HDRCARRY = 8;   // covering frame's header began in the previous batch
constexpr uint32_t S_PARTCARRY = 16; // the carried partial header is still incomplete
constexpr uint32_t S_KEEP = S_NOCOV | S_CARRIED | S_HDRCARRY;

// record layout: R_WORDS x u64 per segment
enum {
  R_META = 0,   // n_entries | n_outcomes << 8 | overflow << 16
  R_ENT0 = 1,   // NENT entries, two per word: pos (16) | rem (13) << 16 | outcome (3) << 29
  R_OUT0 = 9,   // NOUT outcomes x 2 words: exit; cov_ps - ss (20) | hlen (4) << 20 | kw << 32
  R_CI = 25,    // assumed input state (X, cov_ps, cov_start, kw | st << 32)
  R_CO = 29,    // output state computed from it
  R_NA = 33,    // frames whose header starts in the segment (given the input)
  R_NI = 34,    // inclusive frame-count prefix (descriptor ordinals)
  R_HEAD = 35,  // the segment's first 32 bytes as indexed (4 words)
  R_WORDS = 40
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

// Survivors of one indexed segment, kept in LDS until its unmask stage.
struct sv_buf {
  uint32_t pos[SMAX];      // segment-relative position
  uint32_t nrel[SMAX];     // successor position (segment-relative, saturating)
  uint32_t key[SMAX];
  uint16_t jmp[LV][SMAX];  // jmp[b][i]: the 2^b-th successor of i (J_TERM past the chain end)
  uint16_t rem[SMAX];      // frames from this node to the chain end
  uint8_t out[SMAX];       // outcome id / O_* mark
  uint8_t hlen[SMAX];
  uint64_t outs[NOUT][4];  // outcomes: exit, cov_ps, cov_start, kw
  uint64_t seg;
  uint32_t nsurv, overflow;
};

struct __attribute__((aligned(16))) st_lds {
  union {
    uint8_t sub[SUB + HALO];  // index: sub-tile bytes
    fent flist[FCAP];         // unmask: frame list
  };
  uint32_t bits[SUB / 32];    // candidate bitmap of the current sub-tile
  uint16_t nxt[SMAX];         // index: successor survivor / N_EXIT / N_DEAD
  uint16_t last[SMAX];        // index: chain end (T_DEAD: dead end)
  sv_buf sv;
  uint32_t scan[8];
  uint32_t ents[NENT];
  uint32_t bk_n[WIN];         // speculation: exits landing in each window segment
  uint32_t bk[WIN][BKT];
  uint64_t seg_id, chase_X, fbase, nbase;
  cstate in, out;
  uint64_t tstamp;            // wave 0's last s_memtime stamp (stats builds)
  uint32_t nfl, pass_done, nent_pub, nout_pub, mode, node_x, rem_x, red;
};

struct st_params {
  uint8_t* base;
  uint64_t lo, hi, nseg;
  const xyws_carry* cin;  // private snapshot of the incoming carry
  xyws_carry* cout;
  xyws_frame* frames;
  uint64_t cap;
  uint64_t* nframes;
  uint32_t* head;   // [0] ticket, [1] error word, [2] exited workgroups, [3] bad pair seen,
                    // [4..5] u64 frame total
  uint32_t* fA;     // per segment: aggregate published
  uint32_t* fC;     // per segment: (assumed input, output) published
  uint32_t* fN;     // per segment: 1 = count, 2 = inclusive count prefix
  uint32_t* fP;     // per segment: 1 = input == predecessor's output, 2 = not
  uint64_t* recs;   // R_WORDS per segment
  uint32_t opts;
};

// The workgroup's LDS block and the launch parameters, reachable from every
// stage function without passing pointers: a pointer parameter would be a
// generic address, turning every LDS access into a flat instruction that also
// waits on outstanding global loads. Parameters are read through the kernarg
// segment (scalar loads).
__shared__ st_lds g_L;
typedef const __attribute__((address_space(4))) st_params kparams_t;
XYWS_DEV st_params kparams() {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(kparams_t*)(__builtin_amdgcn_kernarg_segment_ptr());
#else
  return st_params{};
#endif
}

// ---------------------------------------------------------------- debug counters
// With XYWS_OPT_STATS the kernel counts resolution events and per-phase
// s_memtime cycles into the stats area (read back by xyws_debug_stats).
enum { ST_EXACT_IN = 0, ST_SPEC, ST_FALLBACK, ST_BADPAIR, ST_REPAIR, ST_MODE1, ST_MODE2,
       ST_NSURV, ST_OVERFLOW, ST_SEGS,
       ST_T_INDEX = 16, ST_T_LINK, ST_T_INPUT, ST_T_CHAIN, ST_T_LIST, ST_T_APPLY,
       ST_F_ISSUE = 24, ST_F_HEAD, ST_F_POLL, ST_F_RECS, ST_F_STAGE0, ST_F_PREAPPLY, ST_F_ACCUM,
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
XYWS_DEV void stat_phase(const st_params& P, uint32_t i, uint64_t& t) {
  if (!stat_on(P)) return;
  const uint64_t now = __builtin_amdgcn_s_memtime();
  stat_add(P, i, now - t);
  t = now;
}
XYWS_DEV void spin_for(const uint32_t* p, uint32_t want, uint32_t* err, uint32_t code) {
  for (uint32_t it = 0; it < SPIN; it++) {
    if (flag_load(p) >= want) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  atomicOr(err, code);
}

// ---------------------------------------------------------------- parsing
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

// Header at absolute position p. Bytes of p's own segment come from global
// memory (a chain's header bytes are never XORed by that chain); bytes past
// the segment end come from the next segment's published first 32 bytes, as
// they were before anyone unmasked that segment.
XYWS_DEV hdr_info header_safe(const st_params& P, uint64_t p) {
  const uint64_t se = (p / SEG + 1) * SEG;
  const uint64_t a = p & ~3ull;
  const uint32_t sh = (uint32_t)(p & 3);
  uint32_t r[5];
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint64_t q = a + 4 * i;
    uint32_t v = 0;
    if (q < P.hi) {
      if (q < se) {
        v = *reinterpret_cast<const uint32_t*>(P.base + q);
      } else {
        const uint64_t w = st_load(P.recs + (se / SEG) * R_WORDS + R_HEAD + ((q - se) >> 3));
        v = (uint32_t)(w >> (((q - se) & 4) * 8));
      }
    }
    r[i] = v;
  }
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
  const uint64_t room = P.hi > p ? P.hi - p : 0;
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

// State before the first byte of the batch (the output of "segment -1"),
// from the carry snapshot.
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

XYWS_DEV const uint64_t* rec_of(const st_params& P, uint64_t k) { return P.recs + k * R_WORDS; }

// Exact chase by header reads from s.X while s.X < lim.
XYWS_DEV void chase_global(const st_params& P, cstate& s, uint64_t lim) {
  const uint64_t stop = lim < P.hi ? lim : P.hi;
  for (;;) {
    if ((s.st & S_PARTIAL) || s.X >= stop) return;
    hdr_info h = header_safe(P, s.X);
    if (!h.hlen) { s.st = (s.st & S_KEEP) | S_PARTIAL; return; }
    s.cov_start = s.X;
    s.cov_ps = s.X + h.hlen;
    s.cov_kw = aligned_key(h.key, s.cov_ps, 0);
    s.X = sat_add(s.cov_ps, h.plen);
    s.cnt++;
    s.st = 0;
  }
}

// ---------------------------------------------------------------- wave/block helpers
XYWS_DEV uint32_t rl32(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
XYWS_DEV uint64_t rl64(uint64_t v, uint32_t l) {
  return ((uint64_t)rl32((uint32_t)(v >> 32), l) << 32) | rl32((uint32_t)v, l);
}
XYWS_DEV void wave_sync() {  // order this wave's LDS accesses across lanes
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
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
  for (uint32_t i = 0; i < NW; i++) {
    const uint32_t si = L.scan[i];
    if (i < wave) wb += si;
    tot += si;
  }
  total = tot;
  return wb + x - v;
}

// ---------------------------------------------------------------- resolution
// Fallback input of segment k (no trusted speculation): the output of the
// nearest segment that has published one, when it is k-1's or reaches k
// (every segment in between is then covered by its last frame); otherwise
// wait for the segments in between.
XYWS_DEV cstate fallback_input(const st_params& P, uint64_t k, uint32_t lane) {
  const uint64_t ts = k * SEG;
  for (uint32_t it = 0; it < SPIN; it++) {
    for (int64_t b = (int64_t)k - 1;; b -= 64) {
      const int64_t j = b - (int64_t)lane;
      const uint32_t fc = j >= 0 ? flag_load(P.fC + j) : (j == -1 ? 1u : 0u);
      const uint64_t m = __ballot(fc >= 1);
      if (!m) continue;  // none of these 64 published: look further back (j = -1 always is)
      const int64_t jj = b - (int64_t)__builtin_ctzll(m);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      cstate S = jj >= 0 ? load_state(rec_of(P, (uint64_t)jj) + R_CO) : initial_state(P);
      S.cnt = 0;
      if (jj == (int64_t)k - 1 || (S.st & S_PARTIAL) || S.X >= ts) return S;
      break;  // a nearer segment continues that chain: wait for it
    }
    __builtin_amdgcn_s_sleep(2);
  }
  atomicOr(P.head + 1, 32u);
  cstate z = initial_state(P);
  z.cnt = 0;
  return z;
}

// Input state of segment k as the whole wave sees it (see the file comment).
// kind: 0 exact, 1 speculated by link support, 2 fallback.
XYWS_DEV cstate resolve_input(const st_params& P, st_lds& L, uint64_t k, uint32_t lane, uint32_t& kind) {
  kind = 0;
  cstate E0 = initial_state(P);
  if (k == 0) return E0;
  const uint64_t ts = k * SEG;
  E0.cnt = 0;
  if ((E0.st & S_PARTIAL) || E0.X >= ts) return E0;  // the batch start reaches k: exact
  const int64_t w0 = (int64_t)k - (int64_t)(WIN - 1);
  const int64_t g = w0 + (int64_t)lane;
  // every window segment was ticketed before k and publishes its aggregate
  // from local work only (long done, one index phase ago)
  bool have = g < 0 || flag_load(P.fA + g) >= 1;
  for (uint32_t it = 0; !__all(have) && it < SPIN; it++) {
    __builtin_amdgcn_s_sleep(1);
    if (!have) have = flag_load(P.fA + g) >= 1;
  }
  if (!__all(have)) atomicOr(P.head + 1, 64u);
  have = have && g >= 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  stat_phase(P, ST_F_POLL, L.tstamp);
  const uint64_t* r = rec_of(P, have ? (uint64_t)g : 0);
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
  if (lane == 0) {  // the batch start's exit supports too
    const int64_t u = (int64_t)(E0.X / SEG) - w0;
    if (E0.X < P.hi && u >= 0 && u < (int64_t)WIN) {
      const uint32_t slot = atomicAdd(&L.bk_n[u], 1u);
      if (slot < BKT) L.bk[u][slot] = (uint32_t)(E0.X - (uint64_t)(w0 + u) * SEG);
    }
  }
  wave_sync();
  stat_phase(P, ST_F_RECS, L.tstamp);
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
  if (!m) {
    kind = 2;
    return fallback_input(P, k, lane);
  }
  kind = 1;
  const uint32_t p = 63 - __builtin_clzll(m);
  const uint64_t pss = (uint64_t)(w0 + (int64_t)p) * SEG;
  const uint64_t w1 = rl64(dW, p);
  cstate I;
  I.cnt = 0;
  I.X = rl64(dX, p);
  I.cov_ps = pss + (w1 & 0xFFFFF);
  I.cov_start = I.cov_ps - ((w1 >> 20) & 0xF);
  I.cov_kw = (uint32_t)(w1 >> 32);
  I.st = 0;
  return I;
}

// Exclusive frame-count prefix of segment k (decoupled look-back sum).
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
    if (lane < li) v = st_load(rec_of(P, (uint64_t)j) + R_NA);
    else if (lane == li && j >= 0) v = st_load(rec_of(P, (uint64_t)j) + R_NI);
#pragma unroll
    for (uint32_t o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);  // lanes > li hold 0
    sum += v;
    if (mi) break;
    b -= 64;
  }
  return sum;
}

// The frames of segment k from input s (lane 0): the path from the entry
// survivor through the jump tables (mode 1), or an exact header chase (mode 2).
struct chain_res {
  cstate o;
  uint32_t mode, node, rem;
};

XYWS_DEV chain_res own_chain(const st_params& P, const sv_buf& S, uint32_t nsurv, uint64_t ss,
                             uint64_t se, const cstate& s) {
  chain_res c;
  c.o = s; c.mode = 0; c.node = 0; c.rem = 0;
  if ((s.st & S_PARTIAL) || s.X >= se || s.X >= P.hi) return c;
  const uint32_t xr = (uint32_t)(s.X - ss);
  uint32_t x = 0, y = nsurv;
  while (x < y) {
    const uint32_t m = (x + y) >> 1;
    if (S.pos[m] < xr) x = m + 1; else y = m;
  }
  if (x < nsurv && S.pos[x] == xr && S.out[x] < NOUT) {
    const uint32_t oc = S.out[x];
    c.mode = 1;
    c.node = x;
    c.rem = S.rem[x];
    c.o.X = S.outs[oc][0]; c.o.cov_ps = S.outs[oc][1]; c.o.cov_start = S.outs[oc][2];
    c.o.cov_kw = (uint32_t)S.outs[oc][3];
    c.o.cnt = s.cnt + c.rem;
    c.o.st = 0;
  } else {
    c.mode = 2;  // the caller chases (chase_global) once seg+1's first bytes are published
  }
  return c;
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

XYWS_DEV __amdgpu_buffer_rsrc_t seg_rsrc(const st_params& P, uint64_t ss) {
  // [ss, ss + round16(hi - ss)) capped at SEG + 16: chunks past the batch read as zero
  const uint64_t room = P.hi - ss;
  const uint32_t nrec = room >= SEG + 16 ? SEG + 16 : (uint32_t)((room + 15) & ~15ull);
  return __builtin_amdgcn_make_buffer_rsrc(P.base + ss, 0, nrec, 0x00020000);
}

// ---------------------------------------------------------------- unmask application
// Frames of segment `seg` from input `sin` (whole workgroup): the covering
// frame, then the path (mode 1, from survivor `node`, `rem` frames) or an exact
// chase (mode 2) in passes of FCAP entries; XOR words accumulate in registers;
// then the changed chunks are loaded, XORed and stored. Descriptors from
// ordinal fb when `emit`.
XYWS_DEV void apply_frames(const st_params& P, st_lds& L, const sv_buf* S, uint64_t seg,
                           const cstate& sin, uint32_t mode, uint32_t node, uint32_t rem, uint64_t fb,
                           bool emit, uint32_t tid, bool stamp = false) {
  const uint64_t ss = seg * SEG, se = ss + SEG, hi = P.hi;
  const bool parse_only = (P.opts & XYWS_OPT_PARSE_ONLY) != 0;
  emit = emit && P.frames;
  __syncthreads();  // the frame list overlays the index stage's sub-tile
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
    const uint32_t base_n = L.nfl;
    for (uint32_t dd = tid; dd < rem; dd += NT) {
      uint32_t i = node;
#pragma unroll
      for (uint32_t bb = 0; bb < LV; bb++)
        if ((dd >> bb) & 1u) i = S->jmp[bb][i];
      const uint64_t p = ss + S->pos[i];
      const uint64_t ps = p + S->hlen[i];
      fent e;
      e.start = S->pos[i];
      e.ps = (uint32_t)(ps - ss);
      e.end = S->nrel[i];
      e.kw = aligned_key(S->key[i], ps, 0);
      L.flist[base_n + dd] = e;
      if (emit) write_frame(P, fb + dd, p, header_safe(P, p), ps, 0);
    }
    __syncthreads();
    if (tid == 0) L.nfl = base_n + rem;
  }
  // Passes of at most FCAP entries. Pass p applies the chunks in [lo_c, hi_c):
  // hi_c = the chunk-aligned start of its last frame (SEG for the final pass);
  // the frames reaching past hi_c carry into the next pass. Every chunk is
  // loaded, XORed and stored once, its loads issued before its XOR words are
  // built.
  const __amdgpu_buffer_rsrc_t rs = seg_rsrc(P, ss);
  const uint32_t voff = tid * 16u;
  const uint64_t lim64 = hi - ss;
  const uint32_t lim = lim64 < SEG ? (uint32_t)lim64 : SEG;  // bytes of this segment in the batch
  uint32_t lo_c = 0;
  for (;;) {
    if (mode == 2 && tid == 0) {  // exact chase, up to FCAP entries per pass
      uint64_t X = L.chase_X, ord = L.fbase;
      uint32_t n = L.nfl;
      const uint64_t stop = se < hi ? se : hi;
      while (X < stop && n < FCAP) {
        hdr_info hh = header_safe(P, X);
        if (!hh.hlen) { X = ~0ull; break; }
        const uint64_t ps = X + hh.hlen;
        fent e;
        e.start = (uint32_t)(X - ss);
        e.ps = (uint32_t)(ps - ss);
        e.end = clamp_rel(sat_add(ps, hh.plen), ss);
        e.kw = aligned_key(hh.key, ps, 0);
        L.flist[n++] = e;
        if (emit) write_frame(P, ord, X, hh, ps, 0);
        ord++;
        X = sat_add(ps, hh.plen);
      }
      L.nfl = n;
      L.fbase = ord;
      L.chase_X = X;
      L.pass_done = !(X < stop);
    }
    __syncthreads();
    const uint32_t nfl = L.nfl;
    const uint32_t done = L.pass_done;
    const uint32_t hi_c = (done || !nfl) ? SEG : (L.flist[nfl - 1].start & ~15u);
    if (!parse_only && nfl) {
      u32x4 d[CHS];
#pragma unroll
      for (uint32_t k = 0; k < CHS; k++) {
        const uint32_t a = (k * NT + tid) * 16u;
        d[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (a >= lo_c && a < hi_c) ? voff : OOB, k * NT * 16u, 0);
      }
      uint32_t g = 0, edge = 0;
#pragma unroll
      for (uint32_t k = 0; k < CHS; k++) {
        const uint32_t a = (k * NT + tid) * 16u;  // increases with k: g only moves forward
        while (g + 1 < nfl && L.flist[g + 1].start <= a) g++;
        const u32x4 x = chunk_xor(L, nfl, g, a);
        const bool nz = (x.x | x.y | x.z | x.w) != 0u;
        const bool inr = a >= lo_c && a < hi_c;
        const bool inb = a + 16 <= lim && !(ss == 0 && a < P.lo);
        __builtin_amdgcn_raw_buffer_store_b128(d[k] ^ x, rs, (inr && nz && inb) ? voff : OOB, k * NT * 16u, 0);
        if (inr && nz && !inb) edge |= 1u << k;
      }
      // first/last chunk of the batch: only the caller's bytes (rare, not unrolled)
#pragma nounroll
      while (edge) {
        const uint32_t k = __builtin_ctz(edge);
        edge &= edge - 1;
        const uint32_t a = (k * NT + tid) * 16u;
        uint32_t ge = 0;
        while (ge + 1 < nfl && L.flist[ge + 1].start <= a) ge++;
        const u32x4 x = chunk_xor(L, nfl, ge, a);
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma nounroll
        for (uint32_t t = 0; t < 16; t++) {
          const uint64_t q = ss + a + t;
          const uint8_t kb = (uint8_t)(w[t >> 2] >> (8u * (t & 3u)));
          if (kb && q >= P.lo && q < hi) P.base[q] ^= kb;
        }
      }
    }
    if (stamp && tid < 64 && done) stat_phase(P, ST_F_ACCUM, L.tstamp);
    __syncthreads();
    if (done) break;
    if (tid == 0) {  // carry the frames reaching past hi_c into the next pass
      uint32_t c = nfl;
      while (c > 0 && L.flist[c - 1].end > hi_c) c--;
      for (uint32_t i = c; i < nfl; i++) L.flist[i - c] = L.flist[i];
      L.nfl = nfl - c;
    }
    lo_c = hi_c;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- index stage
XYWS_DEV void index_segment(const st_params& P, st_lds& L, uint64_t seg, uint32_t tid, uint32_t lane,
                            uint32_t wave) {
  sv_buf& S = L.sv;
  const bool want_unmasked = (P.opts & XYWS_OPT_UNMASKED_HINT) != 0;
  const uint64_t lo = P.lo, hi = P.hi;
  const uint64_t ss = seg * SEG;
  uint64_t* rec = P.recs + seg * R_WORDS;

  // ---- 1. loads: the whole segment into registers
  const __amdgpu_buffer_rsrc_t rs = seg_rsrc(P, ss);
  const uint32_t voff = tid * 16u;
  u32x4 d[CHS];
#pragma unroll
  for (uint32_t k = 0; k < CHS; k++) d[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, k * NT * 16u, 0);
  u32x4 halo = {0u, 0u, 0u, 0u};
  if (tid == 0) halo = __builtin_amdgcn_raw_buffer_load_b128(rs, 0, SEG, 0);
  if (tid == 0) { S.nsurv = 0; S.overflow = 0; S.seg = seg; }
  if (wave == 0) stat_phase(P, ST_F_ISSUE, L.tstamp);
  if (tid < 2) {  // the segment's first 32 bytes, for headers straddling into it
    st_store(rec + R_HEAD + 2 * tid, (uint64_t)d[0].x | ((uint64_t)d[0].y << 32));
    st_store(rec + R_HEAD + 2 * tid + 1, (uint64_t)d[0].z | ((uint64_t)d[0].w << 32));
  }
  if (wave == 0) stat_phase(P, ST_F_HEAD, L.tstamp);

  // ---- 1b. per sub-tile: LDS copy, prefilter, candidates -> survivors
#pragma nounroll
  for (uint32_t s = 0; s < NSUB; s++) {
    const uint64_t ts = ss + (uint64_t)s * SUB, te = ts + SUB;
    __syncthreads();  // previous sub-tile (or the previous unmask stage's list) consumed
    // sub-tile s is always d[0 .. CHSUB): the chunk registers shift down by
    // CHSUB after each sub-tile (register moves, no dynamic indexing)
#pragma unroll
    for (uint32_t k = 0; k < CHSUB; k++) *reinterpret_cast<u32x4*>(&L.sub[(k * NT + tid) * 16u]) = d[k];
    if (tid == 0) *reinterpret_cast<u32x4*>(&L.sub[SUB]) = s + 1 < NSUB ? d[CHSUB] : halo;
#pragma unroll
    for (uint32_t k = 0; k + CHSUB < CHS; k++) d[k] = d[k + CHSUB];
    __syncthreads();
    if (s == 0 && wave == 0) stat_phase(P, ST_F_STAGE0, L.tstamp);
    // prefilter: lane owns sub-tile positions [tid*32, tid*32+32)
    const uint32_t p0 = tid * PPL;
    uint32_t cand = 0;
    {
      uint32_t w = *reinterpret_cast<const uint32_t*>(&L.sub[p0]);
#pragma unroll
      for (uint32_t i = 0; i < PPL / 4; i++) {
        const uint32_t wn = *reinterpret_cast<const uint32_t*>(&L.sub[p0 + 4 * i + 4]);
        const uint32_t b1s = (w >> 8) | (wn << 24);  // byte t = byte at position 4i+t+1
        const uint32_t rsv_ok = ~((w & 0x70707070u) + 0x70707070u) & 0x80808080u;
        const uint32_t bad_op = ((w << 5) | ((w & (w >> 1)) << 7)) & 0x80808080u;
        const uint32_t m_ok = (want_unmasked ? ~b1s : b1s) & 0x80808080u;
        const uint32_t c = rsv_ok & ~bad_op & m_ok;
        const uint32_t nib = ((c >> 7) | (c >> 14) | (c >> 21) | (c >> 28)) & 0xFu;
        cand |= nib << (4 * i);
        w = wn;
      }
      const uint64_t st = ts + p0;
      uint32_t m = ~0u;
      if (st + PPL > hi) m = (st >= hi) ? 0 : ((1u << (hi - st)) - 1);
      if (st < lo) m &= (lo - st >= PPL) ? 0 : ~((1u << (lo - st)) - 1);
      cand &= m;
      L.bits[tid] = cand;
    }
    __syncthreads();
    // candidates: the successor must be a candidate too (or lie past the sub-tile)
    uint32_t surv = 0;
    {
      uint32_t m = cand;
      while (m) {
        const uint32_t b = __builtin_ctz(m);
        m &= m - 1;
        const uint32_t prel = p0 + b;
        const uint64_t pabs = ts + prel;
        const uint32_t b0 = L.sub[prel], b1 = L.sub[prel + 1];
        const uint32_t l7 = b1 & 0x7Fu;
        uint64_t nx;
        if (l7 < 126) {  // short form: no further bytes needed
          if ((b0 & 0x08u) && !(b0 & 0x80u)) continue;  // control frame without FIN
          nx = pabs + 2 + 4 * (b1 >> 7) + l7;
        } else {
          hdr_info hh = header_lds(L.sub, prel, pabs, hi);
          if (!plausible(hh, (uint8_t)b1)) continue;
          nx = sat_add(pabs + hh.hlen, hh.plen);
        }
        if (nx > hi) continue;
        if (nx < te) {
          const uint32_t nr = (uint32_t)(nx - ts);
          if (!((L.bits[nr >> 5] >> (nr & 31)) & 1u)) continue;
        }
        surv |= 1u << b;
      }
    }
    // ordered append: block-exclusive scan of per-lane survivor counts
    uint32_t tot;
    const uint32_t r0 = block_scan(L, __popc(surv), lane, wave, tot);
    const uint32_t base_n = S.nsurv;
    const bool fits = base_n + tot <= SMAX;
    if (fits) {
      uint32_t r = base_n + r0;
      uint32_t m = surv;
      while (m) {
        const uint32_t b = __builtin_ctz(m);
        m &= m - 1;
        const uint32_t prel = p0 + b;
        hdr_info hh = header_lds(L.sub, prel, ts + prel, hi);
        S.pos[r] = s * SUB + prel;
        S.nrel[r] = clamp_rel(sat_add(ts + prel + hh.hlen, hh.plen), ss);
        S.key[r] = hh.key;
        S.hlen[r] = (uint8_t)hh.hlen;
        r++;
      }
    }
    __syncthreads();
    if (tid == 0) {
      if (fits) S.nsurv = base_n + tot;
      else S.overflow = 1;
    }
  }
  __syncthreads();
  if (wave == 0) stat_phase(P, ST_T_INDEX, L.tstamp);

  // ---- 2. link survivors
  const uint32_t nsurv = S.overflow ? 0u : S.nsurv;
  for (uint32_t i = tid; i < nsurv; i += NT) {
    const uint32_t nr = S.nrel[i];
    uint16_t nn = N_EXIT;
    if (nr < SEG) {
      uint32_t x = i + 1, y = nsurv;  // successor lies after i: search (i, nsurv)
      while (x < y) {
        const uint32_t m = (x + y) >> 1;
        if (S.pos[m] < nr) x = m + 1; else y = m;
      }
      nn = (x < nsurv && S.pos[x] == nr) ? (uint16_t)x : N_DEAD;
    }
    L.nxt[i] = nn;
    S.jmp[0][i] = (nn == N_EXIT || nn == N_DEAD) ? J_TERM : nn;
    S.rem[i] = 1;
    L.last[i] = nn == N_EXIT ? (uint16_t)i : (nn == N_DEAD ? T_DEAD : 0);
  }
  __syncthreads();

  // ---- 2a. pointer doubling: after round b, rem/last are final for chains of
  // up to 2^(b+1) nodes and jmp[b+1] holds the 2^(b+1)-th successors
  for (uint32_t b = 0; b < LV; b++) {
    uint32_t nj[NPT], nr[NPT], nl[NPT];
    bool any = false;
#pragma unroll
    for (uint32_t h = 0; h < NPT; h++) {
      const uint32_t i = tid + h * NT;
      nj[h] = J_TERM; nr[h] = 0; nl[h] = 0;
      if (i < nsurv) {
        const uint32_t j = S.jmp[b][i];
        nr[h] = S.rem[i];
        nl[h] = L.last[i];
        if (j != J_TERM) {
          const uint32_t jj = b + 1 < LV ? S.jmp[b][j] : J_TERM;
          nj[h] = jj;
          nr[h] += S.rem[j];
          nl[h] = L.last[j];
          any = any || jj != J_TERM;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t h = 0; h < NPT; h++) {
      const uint32_t i = tid + h * NT;
      if (i < nsurv) {
        if (b + 1 < LV) S.jmp[b + 1][i] = (uint16_t)nj[h];
        S.rem[i] = (uint16_t)nr[h];
        L.last[i] = (uint16_t)nl[h];
      }
    }
    const bool more = __syncthreads_or(any);
    if (!more) {  // every chain resolved: the remaining levels are all J_TERM
      for (uint32_t bb = b + 2; bb < LV; bb++)
        for (uint32_t i = tid; i < nsurv; i += NT) S.jmp[bb][i] = J_TERM;
      break;
    }
  }
  // outcome ids: chain-end nodes ranked in position order (thread tid owns
  // nodes NPT*tid .. NPT*tid+NPT-1)
  {
    uint32_t isl[NPT], nl = 0;
#pragma unroll
    for (uint32_t h = 0; h < NPT; h++) {
      const uint32_t i = NPT * tid + h;
      isl[h] = (i < nsurv && L.nxt[i] == N_EXIT) ? 1u : 0u;
      nl += isl[h];
    }
    uint32_t tot;
    uint32_t id = block_scan(L, nl, lane, wave, tot);
#pragma unroll
    for (uint32_t h = 0; h < NPT; h++) {
      const uint32_t i = NPT * tid + h;
      if (isl[h]) {
        S.out[i] = id < NOUT ? (uint8_t)id : O_UNREC;
        if (id < NOUT) {
          const uint64_t pp = ss + S.pos[i];
          const uint64_t ps = pp + S.hlen[i];
          S.outs[id][0] = S.nrel[i] == 0xFFFFFFFFu ? ~0ull : ss + S.nrel[i];
          S.outs[id][1] = ps;
          S.outs[id][2] = pp;
          S.outs[id][3] = aligned_key(S.key[i], ps, 0);
        }
        id++;
      }
    }
    if (tid == 0) L.nout_pub = tot < NOUT ? tot : NOUT;
    __syncthreads();
    // every node's outcome = its chain end's; entries = the first NENT exiting nodes
    uint32_t ex[NPT], ne = 0;
    uint8_t oc[NPT];
#pragma unroll
    for (uint32_t h = 0; h < NPT; h++) {
      const uint32_t i = NPT * tid + h;
      oc[h] = O_DEAD;
      if (i < nsurv) {
        const uint32_t t = L.last[i];
        oc[h] = t == T_DEAD ? O_DEAD : S.out[t];
      }
      ex[h] = oc[h] < NOUT ? 1u : 0u;
      ne += ex[h];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t h = 0; h < NPT; h++) {
      const uint32_t i = NPT * tid + h;
      if (i < nsurv) S.out[i] = oc[h];
    }
    uint32_t q = block_scan(L, ne, lane, wave, tot);
#pragma unroll
    for (uint32_t h = 0; h < NPT; h++) {
      const uint32_t i = NPT * tid + h;
      if (ex[h]) {
        if (q < NENT) L.ents[q] = S.pos[i] | ((uint32_t)S.rem[i] << 16) | ((uint32_t)oc[h] << 29);
        q++;
      }
    }
    if (tid == 0) L.nent_pub = tot < NENT ? tot : NENT;
  }
  __syncthreads();

  // ---- 3. publish the aggregate: lanes store words in parallel, one drain, one flag
  if (wave == 0) {
    const uint32_t nent = L.nent_pub, nout = L.nout_pub;
    if (lane == 0)
      st_store(rec + R_META, (uint64_t)nent | ((uint64_t)nout << 8) | ((uint64_t)S.overflow << 16));
    if (lane < (nent + 1) / 2) {
      const uint32_t q = 2 * lane;
      st_store(rec + R_ENT0 + lane, (uint64_t)L.ents[q] | (q + 1 < nent ? (uint64_t)L.ents[q + 1] << 32 : 0));
    }
    if (lane >= 16 && lane < 16 + nout) {
      const uint32_t o = lane - 16;
      st_store(rec + R_OUT0 + 2 * o, S.outs[o][0]);
      st_store(rec + R_OUT0 + 2 * o + 1, (S.outs[o][1] - ss) | ((S.outs[o][1] - S.outs[o][2]) << 20) |
                                             (S.outs[o][3] << 32));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(P.fA + seg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (stat_on(P)) {
      stat_add(P, ST_NSURV, nsurv);
      if (S.overflow) stat_add(P, ST_OVERFLOW, 1);
    }
    stat_phase(P, ST_T_LINK, L.tstamp);
  }
}

// ---------------------------------------------------------------- unmask stage
// Steps 4-5 for the lagged segment (wave 0): input state, own frames, and the
// (input, output, count) record stores — issued, not waited for. Runs inside
// the next index stage, while that stage's segment loads are in flight.
XYWS_DEV void resolve_segment(const st_params& P, st_lds& L, uint32_t lane) {
  const sv_buf& S = L.sv;
  const uint64_t seg = S.seg, ss = seg * SEG, se = ss + SEG;
  const uint32_t nsurv = S.overflow ? 0u : S.nsurv;
  uint32_t kind;
  const cstate I = resolve_input(P, L, seg, lane, kind);
  stat_phase(P, ST_T_INPUT, L.tstamp);
  if (lane == 0) {
    const chain_res c = own_chain(P, S, nsurv, ss, se, I);
    if (c.mode != 2) {
      uint64_t* rec = P.recs + seg * R_WORDS;
      store_state(rec + R_CI, I);
      store_state(rec + R_CO, c.o);
      st_store(rec + R_NA, c.o.cnt);
    }
    L.in = I;
    L.out = c.o;
    L.mode = c.mode;
    L.node_x = c.node;
    L.rem_x = c.rem;
    if (stat_on(P)) {
      stat_add(P, kind == 0 ? ST_EXACT_IN : kind == 1 ? ST_SPEC : ST_FALLBACK, 1);
      stat_add(P, c.mode == 2 ? ST_MODE2 : ST_MODE1, 1);
      stat_add(P, ST_SEGS, 1);
    }
  }
  stat_phase(P, ST_T_CHAIN, L.tstamp);
}

// Step 6 (whole workgroup), after resolve_segment: descriptor ordinals (only
// when descriptors are wanted), XOR application, then the (input, output)
// flag and the frame count.
XYWS_DEV void unmask_segment(const st_params& P, st_lds& L, uint32_t tid, uint32_t lane, uint32_t wave) {
  const sv_buf& S = L.sv;
  const uint64_t seg = S.seg;
  uint64_t* rec = P.recs + seg * R_WORDS;
  if (tid == 0 && (P.frames || L.mode == 2)) {
    // header reads (exact chase, descriptors) may straddle into seg+1: its
    // first bytes must be published (its index stage precedes ours: no cycle)
    if (seg + 1 < P.nseg) spin_for(P.fA + seg + 1, 1u, P.head + 1, 2u);
    if (L.mode == 2) {
      cstate o = L.in;
      chase_global(P, o, (seg + 1) * SEG);
      L.out = o;
      store_state(rec + R_CI, L.in);
      store_state(rec + R_CO, o);
      st_store(rec + R_NA, o.cnt);
    }
  }
  if (P.frames && wave == 0) {
    if (lane == 0) flag_publish(P.fN + seg, 1u);
    const uint64_t nbase = count_prefix(P, seg, lane);
    if (lane == 0) {
      st_store(rec + R_NI, nbase + L.out.cnt);
      flag_publish(P.fN + seg, 2u);
      L.nbase = nbase;
    }
  } else if (tid == 0) {
    L.nbase = 0;
  }
  __syncthreads();
  const cstate sin = L.in;
  // the carried-header frame of the batch is described by segment 0
  if (seg == 0 && tid == 0 && (sin.st & S_HDRCARRY) && !(sin.st & S_PARTIAL)) {
    hdr_info hh = header_carried(P.base, P.lo, P.hi, P.cin);
    write_frame(P, 0, P.lo, hh, sin.cov_ps, (int32_t)P.cin->hdr_len);
  }
  if (wave == 0) stat_phase(P, ST_F_PREAPPLY, L.tstamp);
  apply_frames(P, L, &S, seg, sin, L.mode, L.node_x, L.rem_x, L.nbase + sin.cnt, true, tid, true);
  if (wave == 0) stat_phase(P, ST_T_APPLY, L.tstamp);
  if (tid == 0) {
    __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(P.head + 4), L.out.cnt, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    flag_publish(P.fC + seg, 1u);  // (input, output) for fallback inputs of later segments
  }
}

// ---------------------------------------------------------------- finish
// First segment >= from whose pair failed (nseg if none); whole workgroup.
XYWS_DEV uint64_t next_bad(const st_params& P, st_lds& L, uint64_t from, uint32_t tid) {
  __syncthreads();
  if (tid == 0) L.red = 0xFFFFFFFFu;
  __syncthreads();
  for (uint64_t b = from; b < P.nseg; b += NT) {
    const uint64_t j = b + tid;
    const bool bad = j < P.nseg && flag_load(P.fP + j) == 2u;
    if (bad) atomicMin(&L.red, (uint32_t)j);
    if (__syncthreads_or(bad)) break;
  }
  const uint32_t r = L.red;
  __syncthreads();
  return r == 0xFFFFFFFFu ? P.nseg : r;
}

// Descriptors of segment j from its (exact) input at ordinal base fb (lane 0).
XYWS_DEV void emit_segment(const st_params& P, uint64_t j, const cstate& I, uint64_t fb) {
  const uint64_t se = (j + 1) * SEG, stop = se < P.hi ? se : P.hi;
  uint64_t X = I.X, ord = fb;
  if (I.st & S_PARTIAL) return;
  while (X < stop && ord < P.cap) {
    hdr_info hh = header_safe(P, X);
    if (!hh.hlen) return;
    const uint64_t ps = X + hh.hlen;
    write_frame(P, ord++, X, hh, ps, 0);
    X = sat_add(ps, hh.plen);
  }
}

// The last workgroup to exit: repair mis-speculated segments, then the frame
// count and the carry out. Whole workgroup; every other workgroup has exited
// (its stores written back by its release fence).
XYWS_DEV void finish(const st_params& P, st_lds& L, uint32_t tid) {
  const uint64_t nseg = P.nseg;
  int64_t delta = 0;
  cstate E = load_state(rec_of(P, nseg - 1) + R_CO);
  if (flag_load(P.head + 3)) {  // some pair failed: repair in order from the first
    uint64_t k = next_bad(P, L, 1, tid);
    if (k < nseg) E = load_state(rec_of(P, k - 1) + R_CO);
    while (k < nseg) {
      const cstate W = load_state(rec_of(P, k) + R_CI);
      const uint64_t old_n = st_load(rec_of(P, k) + R_NA);
      const uint64_t fb0 = P.frames ? st_load(rec_of(P, k) + R_NI) - old_n : 0;
      if (same_state(W, E)) {  // k's input is exact again: outputs stand until the next bad pair
        const uint64_t nk = next_bad(P, L, k + 1, tid);
        if (delta != 0 && P.frames && tid == 0) {  // ordinals shifted: rewrite their descriptors
          for (uint64_t j = k; j < nk; j++) {
            const uint64_t nj = st_load(rec_of(P, j) + R_NA);
            const uint64_t fbj = st_load(rec_of(P, j) + R_NI) - nj + (uint64_t)delta;
            if (fbj >= P.cap) break;
            emit_segment(P, j, load_state(rec_of(P, j) + R_CI), fbj);
          }
        }
        if (nk >= nseg) { E = load_state(rec_of(P, nseg - 1) + R_CO); break; }
        k = nk;
        E = load_state(rec_of(P, k - 1) + R_CO);
        continue;
      }
      // undo the frames of the wrong input (its chain's header bytes are intact)
      if (stat_on(P)) stat_add(P, ST_REPAIR, 1);
      apply_frames(P, L, nullptr, k, W, 2, 0, 0, 0, false, tid);
      __threadfence();
      __syncthreads();
      // redo from the exact input
      if (tid == 0) {
        cstate o = E;
        o.cnt = 0;
        chase_global(P, o, (k + 1) * SEG);
        L.out = o;
      }
      __syncthreads();
      const cstate o = L.out;
      apply_frames(P, L, nullptr, k, E, 2, 0, 0, fb0 + (uint64_t)delta, true, tid);
      __threadfence();
      __syncthreads();
      delta += (int64_t)o.cnt - (int64_t)old_n;
      E = o;
      k++;
    }
  }
  if (tid == 0) {
    const uint64_t total = __hip_atomic_load(reinterpret_cast<uint64_t*>(P.head + 4), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) + (uint64_t)delta;
    const cstate o = E;
    if (P.nframes) *P.nframes = total;
    if (P.cout) {
      const uint64_t lo = P.lo, hi = P.hi;
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
                                                  : header_safe(P, o.cov_start);
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

// ---------------------------------------------------------------- kernels
// One workgroup per segment, in ticket order (so every segment a workgroup
// waits for belongs to a workgroup that started earlier). Straight-line: index,
// resolve (wave 0), unmask. 4 workgroups = 16 waves per CU (<= 128 VGPRs,
// <= 40 KiB LDS each): while some wait on memory or on predecessors, others run.
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4, 4))) k_stream_fused(st_params P) {
  st_lds& L = g_L;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  if (tid == 0) {
    L.seg_id = atomicAdd(P.head, 1u);
    L.tstamp = stat_on(P) ? __builtin_amdgcn_s_memtime() : 0;
  }
  __syncthreads();
  const uint64_t seg = L.seg_id;
  index_segment(P, L, seg, tid, lane, wave);
  if (wave == 0) resolve_segment(P, L, lane);
  __syncthreads();
  unmask_segment(P, L, tid, lane, wave);
}

// Pair checks after the decode: segment k's assumed input against segment
// k-1's output (one thread per pair; the kernel boundary orders the records).
__global__ void __launch_bounds__(256) k_stream_pairs(st_params P) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x + 1;
  if (k >= P.nseg) return;
  const bool ok = same_state(load_state(rec_of(P, k) + R_CI), load_state(rec_of(P, k - 1) + R_CO));
  P.fP[k] = ok ? 1u : 2u;
  if (!ok) {
    atomicOr(P.head + 3, 1u);
    if (stat_on(P)) atomicAdd(reinterpret_cast<unsigned long long*>(P.head + 32) + ST_BADPAIR, 1ull);
  }
}

// Repairs (if any pair failed), the frame count and the carry out.
__global__ void __launch_bounds__(NT) k_stream_finish(st_params P) { finish(P, g_L, threadIdx.x); }

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

constexpr uint64_t HEAD_BYTES = 512;  // [0] ticket .. [5]; [64..128) carry snapshot; [128..384) stats

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

static uint64_t flags_bytes(uint64_t n) { return (4 * n * 4 + 255) & ~255ull; }  // fA fC fN fP

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
  P.fN = fl + 2 * nseg;
  P.fP = fl + 3 * nseg;
  P.recs = reinterpret_cast<uint64_t*>(m + HEAD_BYTES + flags_bytes(s->max_tiles));
  P.opts = opts;
  // Ticket, exit counter, bad-pair word, total and flags zeroed every call (the
  // error word [1] is sticky until read back). The carry is snapshotted first:
  // dev_carry_in may alias dev_carry_out, which the finishing workgroup writes.
  xyws_carry* snap = reinterpret_cast<xyws_carry*>(m + 64);
  if (hipMemsetAsync(P.head + 2, 0, 16, stream) != hipSuccess) return XYWS_ERR_HIP;  // [2..5]
  if (hipMemsetAsync(P.head, 0, 4, stream) != hipSuccess) return XYWS_ERR_HIP;
  if ((opts & XYWS_OPT_STATS) && hipMemsetAsync(m + 128, 0, 256, stream) != hipSuccess) return XYWS_ERR_HIP;
  if (cin) {
    if (hipMemcpyAsync(snap, cin, sizeof(xyws_carry), hipMemcpyDeviceToDevice, stream) != hipSuccess)
      return XYWS_ERR_HIP;
  } else if (hipMemsetAsync(snap, 0, sizeof(xyws_carry), stream) != hipSuccess) {
    return XYWS_ERR_HIP;
  }
  P.cin = snap;
  if (hipMemsetAsync(fl, 0, (4 * nseg * 4 + 15) & ~15ull, stream) != hipSuccess) return XYWS_ERR_HIP;
  hipLaunchKernelGGL(k_stream_fused, dim3((uint32_t)nseg), dim3(NT), 0, stream, P);
  if (nseg > 1)
    hipLaunchKernelGGL(k_stream_pairs, dim3((uint32_t)((nseg - 1 + 255) / 256)), dim3(256), 0, stream, P);
  hipLaunchKernelGGL(k_stream_finish, dim3(1), dim3(NT), 0, stream, P);
  return hipGetLastError() == hipSuccess ? XYWS_OK : XYWS_ERR_HIP;
}
