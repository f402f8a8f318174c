// xyws_lattice.h — the lattice decoder (k_stream_lattice) of xyws_decode_stream,
// included by xyws_stream.hip inside its anonymous namespace (it shares
// run_params, the header readers, initial_state and write_outputs there).
//
// The frame chain of a batch is a linked list (websocket_frame_header.h:305-385:
// frame k+1 starts at start_k + H_k + P_k). In a batch of equal frames (the
// echo of one message size, the c1/c2/c3/c5 bench batches) the list is a
// lattice: X0 + k*F, X0 the first frame start after the carried frame and F
// the size of the frame there. The lattice decoder tests that hypothesis
// everywhere at once instead of walking the list:
//
//  * Segments of SEG bytes: the first round is static (workgroup b takes
//    segments b and b + grid), then claims in batch order from one counter,
//    one claim ahead (the next segment's loads fly while the current one is
//    decoded), every CU streaming to the end of the batch (scripts/bw_probe6,
//    bw_probe7).
//  * A segment's lattice points are checked by one lane each, from the LDS
//    copy of the segment (and the 16 bytes after it): the header there must
//    open a frame of exactly F bytes — or be the batch's last frame (its
//    payload reaches the batch end, or its header is cut by it). The lanes
//    write a table of the segment's frames (payload range, rotated key word);
//    the frame covering the segment's first bytes comes from its header in
//    memory (headers are never written by a decode: in place, only payload
//    bytes change).
//  * By induction from X0 (exact: the batch start and the carry), every
//    lattice point before the first failing one is an exact frame start. A
//    segment publishes its own result (a status word, AGG: its points hold;
//    BRK: one failed, after raising the global failing point LW_BRK) and
//    counts in its 64-segment group. It does not wait for the segments before
//    it: it stores every chunk below the first failing point KNOWN to it —
//    its own, or LW_BRK as read one segment earlier (from one of 64 replicas).
//    Only a workgroup's first segment is gated (and not after a call the
//    lattice decoder finished: XYWS_OPT_LAT_NOGATE): it waits until every
//    earlier segment has decided and reads LW_BRK fresh, so a batch that
//    breaks near its start stores nothing wrong. Every later store is
//    speculative: the workgroup records (segment, lattice index its stores
//    stop at); at its end a workgroup that knew of a failing point waits
//    until every workgroup's loop has ended (LW_LOOPS: the failing point is
//    final then) and undoes its own stores past it, the others dump their
//    list to scratch and the workgroup finishing the call undoes those
//    (lat_undo: XOR is an involution, keys from the headers in memory,
//    which a decode never writes). A workgroup whose list is
//    full (LAT_SLIST) stops speculating: it raises the failing point to the
//    frame before its segment and the run decoder takes the rest.
//  * Each lane XORs its 16-byte chunks with the keys of the (at most two)
//    frames its chunk overlaps: the frame index is arithmetic (a float
//    reciprocal of F with a +-1 fix), no list walk.
//  * The first failing point kb (a size change, an irregular stream): bytes
//    before X0 + kb*F are decoded and stored, bytes from there on are left
//    as they are, and the workgroup finishing the call writes a redirect
//    record; the run decoder launched after it in the same stream
//    (XYWS_OPT_REDIRECT) decodes [X0 + kb*F, hi) as a fresh stream, counting
//    on from frame c0 + kb. When the hypothesis does not apply at all (a
//    batch inside one frame, a first frame under LAT_FMIN bytes, a header cut
//    by the batch start) the run decoder decodes the whole batch; when the
//    lattice held everywhere it exits at once.
//
// Any byte stream decodes exactly as the reference parses it; the hypothesis
// decides speed only.

constexpr uint64_t LAT_FMIN = 128;          // smaller frames: the run decoder (its dense pass)
constexpr uint64_t LAT_FMAX = 1ull << 40;   // (lattice arithmetic stays well inside 64 bits)
// lattice scratch (u64 words, zeroed at allocation)
enum {
  LW_CNT = 0,      // u32 [0] claim counter, u32 [1] done count (reset by the finisher)
  LW_BRK = 2,      // ~(earliest failing lattice index) of this call, 0 = none (reset by the finisher)
  LW_UNMASK = 3,   // xyws_unmask's claim counter pair (u32 claims, u32 done; reset by its last workgroup)
  LW_W = 4,        // the decided prefix: every segment below it has published its result (reset by the finisher)
  LW_LOOPS = 5,    // workgroups whose segment loop has ended (reset by the finisher)
  // one 16-byte granule, loaded by the prologue in one round trip:
  LW_DPOL = 6,     // the device policy word of the previous call in the stream (dpol_publish)
  LW_EPOCH = 7,    // completed calls (a call runs with E = this + 1)
  LW_REDIR = 8,    // redirect record for the run decoder: [0] state, [1] p, [2] frames before p
  LW_NBAIL_POL = 12,  // calls handed whole to the run decoder on the device policy word (cumulative)
  LW_NBAIL_HYP = 13,  // calls handed whole to the run decoder by the prologue's checks (cumulative)
  LW_NLOOP_A = 14,    // calls whose segment loops ran in the large-frame geometry (cumulative)
  LW_NLOOP_B = 15,    // ... in the default geometry (cumulative)
  LW_RCARRY = 16,  // the carry the run decoder starts from at p (8 words)
  LW_STAT = 32     // per segment: (E << 2) | LS_*
};
enum { LS_AGG = 1, LS_BRK = 3 };
constexpr uint32_t LAT_SLIST = 512;            // speculative stores a workgroup records (lat_undo's list)
constexpr uint32_t LAT_NOCLAIM = 0x7FFFFFFFu;  // (no claim: the next segment after it is none)
enum : uint64_t { RD_DONE = 0, RD_FULL = 1, RD_FROM = 2 };

template <uint32_t NT_, uint32_t SEG_>
struct lgeom {
  static constexpr uint32_t NT = NT_, SEG = SEG_;
  static constexpr uint32_t TMAX = SEG_ / LAT_FMIN + 3;  // covering frame + lattice points
};
// 120 KiB segments: 8 rows of 1 KiB for each of the 15 data waves (wave 0 is
// the control wave; no partial last round: every data wave's loads and stores
// are unconditional), one 1024-thread workgroup per CU
using G_LAT = lgeom<1024, 15 * 8 * 1024>;
// 75 KiB segments (5 rows per data wave): the geometry for frames of 16 KiB
// and more (c3: 0.670 vs 0.688 ms in 120 KiB segments, same box, r05l; rows
// per data wave 3..8 swept in profiles/r05_lattice_rows_ab.txt; c1/c2
// measured no faster in them). One kernel holds both loops and takes one by
// the size of THIS call's first frame (the prologue's F), so the choice never
// lags behind calls in flight.
using G_LAT5 = lgeom<1024, 15 * 5 * 1024>;
constexpr uint64_t LAT5_MIN_FRAME = 16384;
using G_LAT_SMALL = lgeom<64, 1024>;  // tests: 1 KiB segments, many segment boundaries

// The LDS layout of a kernel holding the loops of geometries GA and GB: the
// larger segment and table (the scalar words first: the prologue writes them
// before it knows which loop runs).
static_assert(LW_DPOL == LW_DPOL_WORD && LW_EPOCH == LW_DPOL + 1 && LW_DPOL % 2 == 0, "one 16-byte granule");

template <class GA, class GB>
struct llay {
  static_assert(GA::NT == GB::NT, "one workgroup size");
  static constexpr uint32_t NT = GA::NT;
  static constexpr uint32_t SEG = GA::SEG > GB::SEG ? GA::SEG : GB::SEG;
  static constexpr uint32_t TMAX = GA::TMAX > GB::TMAX ? GA::TMAX : GB::TMAX;
};
template <class GL>
struct __attribute__((aligned(256))) lat_lds {
  cstate S0;                 // the state at the batch start (carry)
  uint64_t E, X0, F, kmax, c0, kbf, nseg;
  uint64_t gk;  // ~(the failing lattice index known to the control wave), 0 = none
  uint32_t na, cur, nxt, brk, quit, done_last, nsl, big, nogate;
  // speculatively stored segments of this workgroup and the lattice index
  // their stores stop at (checked once every earlier segment has decided)
  uint64_t sl_seg[LAT_SLIST], sl_k[LAT_SLIST];
  uint4 tab[GL::TMAX];        // frames overlapping the segment: {ps, end, kw, 0} segment-relative
  // the segment, the 16 bytes after it, and the 20 bytes at the dword at or
  // below the header of the frame covering its first bytes (256-byte aligned:
  // the rows' LDS bank pattern does not depend on the table's size)
  alignas(256) uint8_t seg[GL::SEG + 48];
};

// Segment-relative clamp of an absolute position to [0, 2^32).
XYWS_DEV uint32_t lat_rel(uint64_t x, uint64_t ss) {
  if (x <= ss) return 0;
  const uint64_t d = x - ss;
  return d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
}

// Segments per decided-prefix group: a segment adds one to its group's
// counter (P.lgrp, reset by the finisher) after publishing its result, so a
// full counter says 64 segments decided in one load.
constexpr uint32_t LAT_GRP = 64;
XYWS_DEV uint64_t lat_grp_size(const run_params& P, uint64_t g) {
  const uint64_t a = g * LAT_GRP;
  return a >= P.nseg ? 0 : (P.nseg - a < LAT_GRP ? P.nseg - a : LAT_GRP);
}

// The decided prefix (wave 0, every lane; the result in every lane): from
// LW_W on, the full groups (64 counters at once: 4096 segments), then the
// segments of the next group (4 statuses per lane: 256), raising LW_W past
// what is decided. Ordering without fences (an agent-scope release fence is
// a write-back of the XCD's whole L2 on gfx950, buffer_wbl2 sc1): every word
// here is read and written at the coherence point (agent-scope atomics, sc1),
// and each operation is issued after the one it depends on has completed — a
// segment raises LW_BRK with a returning atomic before it publishes its
// result and counts in its group, the raise of LW_W follows the loads of the
// results it covers, and a reader of LW_W loads LW_BRK after it — so a
// workgroup that sees LW_W > s reads in LW_BRK every failing point of
// segments <= s.
XYWS_DEV uint64_t lat_advance(const run_params& P, uint64_t E, uint32_t lane) {
  const uint64_t w = uniform64(st_load(P.lat + LW_W));
  if (w >= P.nseg) return w;
  uint64_t w1 = w;
  {
    const uint64_t g0 = w / LAT_GRP, g = g0 + lane, gs = lat_grp_size(P, g);
    const bool full = !gs || st_load(P.lgrp + g) == gs;
    const uint64_t nf = __ballot(!full);
    const uint32_t c = nf ? (uint32_t)__builtin_ctzll(nf) : 64u;
    const uint64_t wg = (g0 + c) * LAT_GRP;
    if (wg > w1) w1 = wg < P.nseg ? wg : P.nseg;
  }
  if (w1 < P.nseg) {
    bool dec[4];
#pragma unroll
    for (uint32_t r = 0; r < 4; r++) {
      const uint64_t j = w1 + 4 * lane + r;
      dec[r] = j >= P.nseg || (st_load(P.lat + LW_STAT + j) >> 2) == E;
    }
    // the lane's first undecided status, then the first lane with one
    const uint32_t lc = !dec[0] ? 0u : !dec[1] ? 1u : !dec[2] ? 2u : !dec[3] ? 3u : 4u;
    const uint64_t nd = __ballot(lc < 4);
    uint64_t w2 = w1 + 256;
    if (nd) {
      const uint32_t f = (uint32_t)__builtin_ctzll(nd);
      w2 = w1 + 4 * f + (uint32_t)__shfl((int)lc, (int)f, 64);
    }
    w1 = w2 < P.nseg ? w2 : P.nseg;
  }
  if (w1 > w && lane == 0) __hip_atomic_fetch_max(P.lat + LW_W, w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return w1;
}
// Wait (wave 0) until every segment up to s has decided; bounded (device
// error bit 2). Every segment at or below s was claimed by a running
// workgroup and decides on its own bytes, so the wait ends.
XYWS_DEV void lat_wait_decided(const run_params& P, uint64_t E, uint64_t s, uint32_t lane) {
  for (uint32_t it = 0; lat_advance(P, E, lane) <= s; it++) {
    if (it >= (1u << 20)) {
      if (lane == 0) atomicOr(P.head + 1, 2u);
      return;
    }
    __builtin_amdgcn_s_sleep(8);  // (polls at the coherence point: spaced)
  }
}

// XOR mask of the 16-byte chunk at segment offset a from the table: entry
// `idx` and the one after it (a chunk meets at most two frames, F >= 16).
// (every wave of a small-frame batch takes the second form on some lane: a
// chunk meeting a frame boundary or a header; span_key16 keeps it short)
XYWS_DEV u32x4 lat_mask(const uint4* tab, uint32_t nent, uint32_t idx, uint32_t a) {
  const uint4 g = tab[idx];
  if (g.x <= a && a + 16u <= g.y) return u32x4{g.z, g.z, g.z, g.z};
  u32x4 m = span_key16(a, g.x, g.y, g.z);
  if (idx + 1 < nent) {
    const uint4 n = tab[idx + 1];
    if (n.x < a + 16u) m |= span_key16(a, n.x, n.y, n.z);
  }
  return m;
}

// The header at segment offset xr (absolute x) from the LDS copy of the
// segment and the 16 bytes after it, cut at the batch end.
XYWS_DEV hdr_info lat_hdr(const run_params& P, const uint8_t* seg, uint32_t xr, uint64_t x) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(seg + (xr & ~3u));
  const uint32_t sh = xr & 3u, r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
  uint32_t w[4];
  w[0] = __builtin_amdgcn_alignbyte(r1, r0, sh);
  w[1] = __builtin_amdgcn_alignbyte(r2, r1, sh);
  w[2] = __builtin_amdgcn_alignbyte(r3, r2, sh);
  w[3] = __builtin_amdgcn_alignbyte(r4, r3, sh);
  const uint64_t room = P.hi - x;
  return parse_header_words(w, room < 16 ? (uint32_t)room : 16u);
}

// Buffer resource over [ss, ss + n) cut at round16(hi): loads past it read
// zero, stores past it are dropped.
XYWS_DEV __amdgpu_buffer_rsrc_t lat_rsrc(const run_params& P, uint64_t ss, uint32_t n) {
  const uint64_t top = (P.hi + 15) & ~15ull;
  const uint64_t room = top > ss ? top - ss : 0;
  return __builtin_amdgcn_make_buffer_rsrc(P.base + ss, 0, room < n ? (uint32_t)room : n, 0x00020000);
}

XYWS_DEV void write_frame(const run_params& P, uint64_t ord, uint64_t start, const hdr_info& h, uint64_t ps,
                          int32_t hdr_shift);

// The descriptor of the frame whose header began in the previous batch
// (frame 0 of the call), as k_stream_emit writes it.
XYWS_DEV void lat_carried_frame(const run_params& P, const xyws_carry* cz) {
  if (!P.frames || !P.cap || cz->payload_remaining || !cz->hdr_len) return;
  const hdr_info hh = header_carried(P, cz);
  if (hh.hlen) write_frame(P, 0, P.lo, hh, P.lo + (hh.hlen - cz->hdr_len), (int32_t)cz->hdr_len);
}

// The workgroup that finished the call last (lane 0; every other workgroup
// has exited): the call's outputs when every lattice point held, else the
// redirect record for the run decoder launched after this kernel; then the
// counters are reset and the epoch advances.
template <class LL>
XYWS_DEV void lat_finish(const run_params& P, LL& L) {
  uint64_t* rd = P.lat + LW_REDIR;
  const xyws_carry* cz = P.cin_user ? P.cin_user : &k_zero_carry;
  {
    const uint32_t w = L.na == 2 ? LW_NBAIL_POL : L.na ? LW_NBAIL_HYP : L.big ? LW_NLOOP_A : LW_NLOOP_B;
    st_store(P.lat + w, st_load(P.lat + w) + 1);
  }
  if (L.na) {
    st_store(rd, RD_FULL);  // the run decoder decodes the whole batch
  } else {
    const uint64_t b = st_load(P.lat + LW_BRK);
    const uint64_t X0 = L.X0, F = L.F, kmax = L.kmax, c0 = L.c0;
    lat_carried_frame(P, cz);
    if (b) {
      // the first failing point is an exact frame start (every point before
      // it held): the run decoder takes the batch from there as a fresh
      // stream, counting on from the frames before it
      const uint64_t kb = ~b;
      const uint64_t tb = c0 + kb;
      uint64_t* rc = P.lat + LW_RCARRY;
#pragma unroll
      for (int i = 0; i < 8; i++) st_store(rc + i, 0);
      st_store(rc + 2, cz->frames_total + tb);
      st_store(rd + 1, X0 + kb * F);
      st_store(rd + 2, tb);
      st_store(rd, RD_FROM);
    } else {
      // every point held: the last lattice point ends the chain
      const uint64_t xl = X0 + (kmax - 1) * F;
      const hdr_info h = hdr_global(P, xl, NONE);
      uint64_t total = c0 + kmax;
      cstate S;
      if (!h.hlen) {  // a header cut by the batch end: carried
        S.X = xl; S.cov_ps = xl; S.cov_start = xl; S.cov_kw = 0; S.cov_key = 0; S.st = S_PARTIAL | S_NOCOV; S.pad = 0;
        total--;
      } else {
        S = frame_state(xl, h);
      }
      xyws_carry cinc;
#pragma unroll
      for (int i = 0; i < 8; i++) reinterpret_cast<uint64_t*>(&cinc)[i] = reinterpret_cast<const uint64_t*>(cz)[i];
      write_outputs(P, &cinc, total, S);  // (after every read of cz: the carry out may alias it)
      dpol_publish(P, F, DEC_LATTICE);
      if (P.pol) {
        const uint64_t v[5] = {L.E, P.hi - P.lo, F, F, DEC_LATTICE};
#pragma unroll
        for (int i = 1; i < 5; i++) __hip_atomic_store(P.pol + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(P.pol, v[0], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      st_store(rd, RD_DONE);
    }
  }
  uint32_t* cnt = reinterpret_cast<uint32_t*>(P.lat + LW_CNT);
  st_store(P.lat + LW_BRK, 0);
  st_store(P.lat + LW_W, 0);
  st_store(P.lat + LW_LOOPS, 0);
  __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  st_store(P.lat + LW_EPOCH, L.E);
}

// The run decoder and its descriptor kernel launched after the lattice
// decoder (XYWS_OPT_REDIRECT): false when the lattice decoded everything;
// else P is the batch from the first failing point on (a fresh stream whose
// frame count, descriptor ordinals and offsets continue the call's), or the
// whole batch as given. Every workgroup runs it first, with the same result.
XYWS_DEV bool lat_redirect(run_params& P) {
  if (!(P.opts & XYWS_OPT_REDIRECT)) return true;
  const uint64_t* r = P.lat + LW_REDIR;
  const uint64_t st = uniform64(st_load(r));
  if (st == RD_DONE) return false;
  if (st != RD_FROM) return true;
  const uint64_t p = uniform64(st_load(r + 1)), tb = uniform64(st_load(r + 2));
  const uint64_t pal = p & ~15ull;
  P.obias = p - P.lo;
  P.base += pal;
  P.lo = p - pal;
  P.hi -= pal;
  // runs over the rest, cut as stream_decode_fused cuts a batch, with the
  // launched run count as the cap
  const uint64_t seg = P.segb, nseg = (P.hi + seg - 1) / seg, maxr = P.nruns;
  P.rbytes = nseg <= maxr ? seg : ((P.hi + maxr - 1) / maxr + 15) & ~15ull;
  P.nruns = (uint32_t)((P.hi + P.rbytes - 1) / P.rbytes);
  P.nflat = 2 * P.nruns;
  P.cin_user = reinterpret_cast<const xyws_carry*>(P.lat + LW_RCARRY);
  P.tbias = tb;
  if (P.frames) {
    const uint64_t c = P.cap < tb ? P.cap : tb;
    P.frames += c;
    P.cap -= c;
  }
  return true;
}

// Roles (round 3's sweep decoder, retired, had the same split): in the production geometry wave
// 0 is the CONTROL wave — claims, the covering frame's header and the 16 bytes
// after the segment (loaded one segment ahead), the published results and the
// look-back — and never loads or stores segment bytes, so its memory
// operations never wait behind a segment's loads (vmcnt counts a wave's
// operations in issue order); waves 1..15 move the data, one 1 KiB row per
// wave instruction. In the one-wave test geometry wave 0 does both.
template <class G>
struct lat_io {
  static constexpr bool CTRL = G::NT >= 256;
  static constexpr uint32_t NW = G::NT / 64, NDW = CTRL ? NW - 1 : NW;
  static constexpr uint32_t NROW = G::SEG / 1024, K = (NROW + NDW - 1) / NDW;
  static constexpr uint32_t CLAIM = CTRL ? 64u : 0u;  // the claim lane: lane 0 of the first data wave
  static_assert(G::SEG % 1024 == 0, "segments are whole 1 KiB rows");
  XYWS_DEV static bool data_wave(uint32_t wave) { return !CTRL || wave != 0; }
  XYWS_DEV static uint32_t row(uint32_t wave, uint32_t k) { return (CTRL ? wave - 1 : wave) + NDW * k; }
  XYWS_DEV static bool valid(uint32_t wave, uint32_t k) { return K * NDW == NROW || row(wave, k) < NROW; }
};

// An agent-coherent load whose value is used a segment later: inline asm, so
// that the compiler neither waits for it nor counts it (the control wave waits
// for all of its operations at once, a segment later: lat_loop).
XYWS_DEV uint64_t lat_load_late(const uint64_t* p) {
  uint64_t v;
  asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// LW_BRK and its replicas (P.lbrk: LAT_NREP words LAT_REPW apart, each
// workgroup reading one per segment: one word read by every CU at the
// coherence point each segment cost a third of the bandwidth,
// scripts/bw_probe9). Raised (wave 0, every lane) to failing point k: the
// word itself with a returning atomic, then every replica, all completed
// before the caller publishes anything.
constexpr uint32_t LAT_NREP = 64, LAT_REPW = 32;
// (word offset of the replicas in the lattice scratch: after the statuses and
// the group counts, 256-byte aligned)
inline constexpr uint64_t lat_rep_off(uint64_t segs) {
  return (LW_STAT + segs + segs / 64 + 1 + LAT_REPW - 1) / LAT_REPW * LAT_REPW;
}
inline constexpr uint64_t lat_sl_off(uint64_t segs) { return lat_rep_off(segs) + LAT_NREP * LAT_REPW; }
// The replicas only when the word itself moved (a break no earlier than one
// already recorded changes nothing; a replica behind the word costs only
// speculation, every decision that must be exact reads the word).
XYWS_DEV void lat_raise_brk(const run_params& P, uint64_t k, uint32_t lane) {
  uint64_t o = 0;
  if (lane == 0) o = __hip_atomic_fetch_max(P.lat + LW_BRK, ~k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (uniform64(o) >= ~k) return;  // (the returning atomic's wait: the compiler's)
  __hip_atomic_fetch_max(P.lbrk + LAT_REPW * lane, ~k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The claim wave's extra loads for segment s, one dword per lane, issued with
// its rows: lanes 0..3 the 16 bytes after the segment, lanes 4..8 the 20
// bytes at the dword at or below the header of the frame covering the
// segment's first bytes (lattice point ka-1) — lane i's dword goes to
// L.seg[SEG + 4i]. One register (a load into registers
// the compiler also pairs with others made it wait for every load in flight).
// Dwords at or past the batch's last one read that one instead (each address
// stays on the batch's pages; the readers cut at hi).
XYWS_DEV uint32_t lat_ctrl_load(const run_params& P, uint64_t s, uint64_t SEGB, uint64_t X0, uint64_t F, uint64_t kmax,
                                uint32_t tid) {
  const uint64_t ss = s * SEGB;
  const uint64_t ka = ss <= X0 ? 0 : (ss - X0 + F - 1) / F;
  const uint64_t xc = ka && ka <= kmax ? X0 + (ka - 1) * F : ss;
  const uint64_t top = (P.hi + 3) & ~3ull;
  // (lane offsets from the per-segment opaque tid: 32-bit, not hoisted)
  const uint32_t lane = tid & 63u;
  const bool pd = lane < 4;
  uint64_t q = (pd ? ss + SEGB : xc & ~3ull) + (uint32_t)(pd ? 4u * lane : 4u * (lane - 4u));
  if (q + 4 > top) q = top - 4;
  return __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(P.base + q));
}

// The segment loop of one role (lat_io): the control lane's claims, loads,
// results and look-back (ROLE CTRL), the data waves' loads, checks, XOR and
// stores (DATA), or both (ALL: the one-wave geometry). Both loops meet the
// same four barriers per segment (A: LDS free, B: segment in LDS, C: table
// and checks done, D: the look-back's answer), so the control wave's state
// and the data waves' prefetch registers never share a register allocation
// region (one loop holding both spilled the prefetch in round 3's sweep decoder).
enum { LR_ALL = 0, LR_CTRL = 1, LR_DATA = 2 };
// stats mode (XYWS_OPT_STATS): shader clocks summed over workgroups, per phase,
// for the control lane (tid 0) and one data lane (tid 64) — the debug stats
// words from 16 on (the run decoder's timing slots; it does not run in a call
// the lattice finished)
enum { LT_C_A = 16, LT_C_C, LT_C_ADV, LT_D_FILL, LT_D_WB, LT_D_TAB, LT_D_WC, LT_D_MASK, LT_D_WD, LT_D_ST, LT_D_WA,
       LT_SEGS, LT_GATE, LT_END };
struct lat_clock {
  bool on;
  uint64_t t, acc[16];
  XYWS_DEV void start(bool o) {
    on = o;
    for (int i = 0; i < 16; i++) acc[i] = 0;
    t = on ? __builtin_amdgcn_s_memtime() : 0;
  }
  XYWS_DEV void mark(int slot) {
    if (!on) return;
    const uint64_t n = __builtin_amdgcn_s_memtime();
    acc[slot - 16] += n - t;
    t = n;
  }
  XYWS_DEV void flush(const run_params& P) {
    if (!on) return;
    for (int i = 0; i < 16; i++)
      if (acc[i]) stat_add(P, 16 + i, acc[i]);
  }
};
template <class G, int ROLE, class LL>
XYWS_DEV void lat_loop(const run_params& P, LL& L, uint32_t tid0, uint32_t ahead) {
  using IO = lat_io<G>;
  constexpr bool CT = ROLE != LR_DATA, DT = ROLE != LR_CTRL;
  uint32_t tid = tid0;
  asm volatile("" : "+v"(tid));  // (opaque: hipcc would hoist the lane address math per segment and spill it)
  const uint32_t lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(P.lat + LW_CNT);
  const uint64_t E = uniform64(L.E);
  const uint64_t X0 = uniform64(L.X0), F = uniform64(L.F), kmax = uniform64(L.kmax);
  const float rF = 1.0f / (float)(F < (1ull << 24) ? F : (1ull << 24));
  const uint32_t F32 = F < 0x80000000ull ? (uint32_t)F : 0x80000000u;
  uint32_t cur = uniform32(L.cur);
  uint32_t it = 0, nsl = 0;  // segments done; speculative stores recorded (every thread)
  lat_clock clk;
  clk.start(stats_on(P) && (tid == 0 || (tid == 64 && DT)));
  uint64_t brk_seen = 0;                        // control lane: LW_BRK as loaded one segment ago
  const bool cl = tid == 0 && CT;  // (which lane's clock this is: control or data)
  u32x4 e[DT ? IO::K : 1];
  uint32_t cx = 0;  // claim wave: lat_ctrl_load's dword
  constexpr uint32_t CW = IO::CLAIM / 64u;
  // a segment's loads: the claim wave first claims the segment after it (the
  // atomic's value is read a segment later, inline asm: the compiler would
  // wait for it at once) and loads the covering header and the bytes after
  // it; then every data wave its rows, the youngest loads (the fill waits for
  // them, and so for everything before them)
  auto issue = [&](uint32_t s, bool claim, bool rows) {
    if constexpr (DT) {
      if (wave == CW) {
        if (lane == 0) {
          if (claim)
            asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(ahead) : "v"(cnt), "v"(1u) : "memory");
          else
            ahead = LAT_NOCLAIM;
        }
        cx = lat_ctrl_load(P, s, G::SEG, X0, F, kmax, tid);
      }
      if (rows) {
        const __amdgpu_buffer_rsrc_t rs = lat_rsrc(P, (uint64_t)s * G::SEG, G::SEG);
#pragma unroll
        for (uint32_t k = 0; k < IO::K; k++)
          e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, IO::valid(wave, k) ? lane * 16u : OOB,
                                                       IO::row(wave, k) * 1024u, AUX_NT);
      }
    }
  };
  if (DT && cur != NONE32) {
    const uint32_t a0 = ahead;
    issue(cur, false, true);
    ahead = a0;  // (claimed at the start)
    // K dropped stores (out-of-range offset, no traffic) after the first
    // loads, as after every later segment's: the fill's waits then count the
    // stores younger than the loads on every path into the loop
    const __amdgpu_buffer_rsrc_t rs = lat_rsrc(P, (uint64_t)cur * G::SEG, G::SEG);
#pragma unroll
    for (uint32_t k = 0; k < IO::K; k++)
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, rs, OOB, k * 1024u, AUX_ST_STREAM);
  }
  // the data lanes number the lattice points of a segment among themselves
  const uint32_t dl = IO::CTRL ? tid - 64u : tid, NDL = IO::NDW * 64u;
  while (cur != NONE32) {
    asm volatile("" : "+v"(tid));
    const uint64_t ss = (uint64_t)cur * G::SEG;
    const uint64_t se = ss + G::SEG;
    const uint64_t ka = ss <= X0 ? 0 : (ss - X0 + F - 1) / F;
    clk.mark(cl ? LT_C_ADV : LT_D_ST);
    __syncthreads();  // (A) the previous segment's LDS reads are done
    clk.mark(cl ? LT_C_ADV : LT_D_WA);
    if constexpr (DT) {
#pragma unroll
      for (uint32_t k = 0; k < IO::K; k++)
        if (IO::valid(wave, k)) *reinterpret_cast<u32x4*>(&L.seg[IO::row(wave, k) * 1024u + lane * 16u]) = e[k];
      if (clk.on) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (DT && wave == CW) {
      // the claim and the control loads were issued just before this
      // segment's rows: landed with them (a use of the last row's register
      // orders the claim's inline-asm value after that wait)
      asm volatile("" : "+v"(ahead), "+v"(cx) : "v"(e[IO::K - 1].x));
      const uint32_t ln = tid & 63u;  // (from the per-segment opaque tid: not hoisted)
      if (ln < 9) *reinterpret_cast<uint32_t*>(&L.seg[G::SEG + 4u * ln]) = cx;
      if (lane == 0) {
        // (claimed a segment ago: the counter's value, after the static first round)
        const uint32_t a = ahead + 2u * gridDim.x;  // (LAT_NOCLAIM: past every segment)
        L.nxt = a < P.nseg ? a : NONE32;
        L.brk = NONE32;
      }
    }
    clk.mark(cl ? LT_C_A : LT_D_FILL);
    __syncthreads();  // (B)
    clk.mark(cl ? LT_C_A : LT_D_WB);
    const uint32_t nxt = uniform32(L.nxt);
    uint64_t kz = se <= X0 ? 0 : (se - X0 + F - 1) / F;
    if (kz > kmax) kz = kmax;
    const uint32_t nl = kz > ka ? (uint32_t)(kz - ka) : 0u;
    if constexpr (DT) {
      if (tid == IO::CLAIM) {
        // the frame covering the segment's first bytes (entry 0)
        uint4 c = {0u, 0u, 0u, 0u};
        if (ka == 0) {
          const cstate S0 = L.S0;
          if (!(S0.st & S_NOCOV)) c = uint4{lat_rel(S0.cov_ps, ss), lat_rel(X0, ss), S0.cov_kw, 0u};
        } else if (ka <= kmax) {
          const uint64_t xc = X0 + (ka - 1) * F;
          const uint32_t sh = (uint32_t)(xc & 3);
          uint32_t w[4];
          const uint32_t* cw = reinterpret_cast<const uint32_t*>(&L.seg[G::SEG + 16]);
#pragma unroll
          for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(cw[i + 1], cw[i], sh);
          const uint64_t room = P.hi - xc;
          const hdr_info h = parse_header_words(w, room < 16 ? (uint32_t)room : 16u);
          if (h.hlen) {
            const uint64_t ps = xc + h.hlen;
            const uint64_t end = ka == kmax ? sat_add(ps, h.plen) : xc + F;
            c = uint4{lat_rel(ps, ss), lat_rel(end < P.hi ? end : P.hi, ss), aligned_key(h.key, ps, 0), 0u};
          }
        }
        L.tab[0] = c;
      }
      if (nxt != NONE32) issue(nxt, !L.quit, true);  // (in flight through the checks, the look-back and the stores)
      // lattice points in the segment: k in [ka, kz), each checked by one data lane
      const uint32_t nlw = (P.opts & XYWS_OPT_LATX_NOWORK) ? 0u : nl;  // (timing experiment)
      for (uint32_t i = dl; i < nlw; i += NDL) {
        const uint64_t k = ka + i;
        const uint64_t x = X0 + k * F;
        const uint32_t xr = (uint32_t)(x - ss);
        const hdr_info h = lat_hdr(P, L.seg, xr, x);
        const bool last = k + 1 == kmax;
        const uint64_t fend = h.hlen ? sat_add(x + h.hlen, h.plen) : x;
        // the point holds: a frame of exactly F bytes, or the batch's last
        // frame (cut by the batch end, or a header the end cuts)
        const bool ok = h.hlen ? ((uint64_t)h.hlen + h.plen == F && h.plen < F) || (last && fend >= P.hi) : last;
        if (!ok) atomicMin(&L.brk, i);
        uint4 en = {xr, xr, 0u, 0u};
        if (h.hlen) {
          const uint64_t ps = x + h.hlen;
          en = uint4{lat_rel(ps, ss), lat_rel(fend < P.hi ? fend : P.hi, ss), aligned_key(h.key, ps, 0), 0u};
        }
        L.tab[1 + i] = en;
      }
    }
    // (B..C) the control lane: every operation it issued a segment ago (its
    // load of LW_BRK, the status store, the group count) has completed: one
    // wait, then the failing point known from LW_BRK as loaded then (stale by
    // a segment: speculation, checked at the end of the work) for this
    // segment's stores
    if (CT && tid == 0) {
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(brk_seen)::"memory");
      if (cl) clk.mark(LT_GATE);  // (stats: the control wave's wait for its operations of a segment ago)
      L.gk = brk_seen;
    }
    clk.mark(cl ? LT_C_A : LT_D_TAB);
    __syncthreads();  // (C) the table and the segment's own checks are complete
    clk.mark(cl ? LT_C_C : LT_D_WC);
    const uint32_t brk = uniform32(L.brk);
    // the workgroup's first segment waits for every earlier one to decide
    // (they are all in their first segment too: a failing point near the
    // batch start is seen before any store, so a miss stores nothing)
    // (XYWS_OPT_TEST_LATSPEC: no gate and no LW_BRK filter, so that a broken
    // lattice stores past its failing point and the end-of-work check undoes
    // it)
    const bool blind = (P.opts & XYWS_OPT_TEST_LATSPEC) != 0;
    const bool gate = it == 0 && !blind && !(P.opts & XYWS_OPT_LAT_NOGATE);
    if (CT && tid < 64) {
      // the segment's own result, published while the data waves store
      // (completed before the result is published; nothing to raise when an
      // earlier failing point is known already)
      const uint64_t gk = uniform64(L.gk);
      if (brk != NONE32 && !(gk && ~gk <= ka + brk)) lat_raise_brk(P, ka + brk, lane);
      if (tid == 0) {
        st_store(P.lat + LW_STAT + cur, (E << 2) | (brk != NONE32 ? LS_BRK : LS_AGG));
        __hip_atomic_fetch_add(P.lgrp + cur / LAT_GRP, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (gate) {
        const uint64_t tg = clk.on ? __builtin_amdgcn_s_memtime() : 0;
        lat_wait_decided(P, E, cur, lane);
        if (tg && tid == 0) stat_add(P, LT_END, __builtin_amdgcn_s_memtime() - tg);  // (stats: the gate's wait)
        if (tid == 0) L.gk = st_load(P.lat + LW_BRK);
      }
      // the load for the next segment's decision (the last operation of the
      // phase: used a segment later)
      if (tid == 0) brk_seen = lat_load_late(P.lbrk + LAT_REPW * (blockIdx.x % LAT_NREP));
    }
    if (gate) __syncthreads();  // (D, the first segment only) the fresh failing point
    clk.mark(cl ? LT_C_C : LT_D_WD);
    // where the segment's stores stop: its own failing point or an earlier
    // one known (every thread: the same uniform arithmetic)
    const uint64_t b = blind ? 0 : uniform64(L.gk);
    uint64_t kst = brk != NONE32 ? ka + brk : kz;
    if (b && ~b < kst) kst = ~b;
    uint32_t stop = kst >= kz ? G::SEG : lat_rel(X0 + kst * F, ss);  // (kst <= kmax: inside the lattice's span)
    if (stop > G::SEG) stop = G::SEG;
    bool quit = b || brk != NONE32;  // the rest of the batch is the run decoder's
    // a store not known valid now is checked at the end (gate: known)
    if (stop && !gate) {
      if (nsl < LAT_SLIST) {
        if (tid == IO::CLAIM) {
          L.sl_seg[nsl] = cur;
          L.sl_k[nsl] = kst;
        }
        nsl++;
      } else {
        // (the list is full: no more speculation here; the lattice stops
        // before this segment's first frame and the run decoder takes the
        // rest, stores past it being undone as any others)
        const uint64_t k0 = ka ? ka - 1 : 0;
        if (tid == IO::CLAIM)
          for (uint32_t r = 0; r <= LAT_NREP; r++)
            __hip_atomic_fetch_max(r < LAT_NREP ? P.lbrk + LAT_REPW * r : P.lat + LW_BRK, ~k0, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (k0 < kst) {
          stop = lat_rel(X0 + k0 * F, ss);
          kst = k0;
        }
        quit = true;
      }
    }
    if (quit && tid == IO::CLAIM) L.quit = 1;  // (read at the next segment's claim)
    if constexpr (DT) {
      // stores: each chunk XORed with the keys of the (at most two) frames it
      // overlaps (a frame's header bytes get a zero mask), every chunk below
      // the failing point known
      const uint32_t xka = ka < kmax ? lat_rel(X0 + ka * F, ss) : 0xFFFFFFFFu;  // first lattice point (relative)
      const uint32_t nent = brk != NONE32 ? 1u + brk : 1u + nl;
      const uint32_t lo_r = lat_rel(P.lo, ss), hi_r = P.hi - ss < G::SEG ? (uint32_t)(P.hi - ss) : G::SEG;
      const __amdgpu_buffer_rsrc_t rs = lat_rsrc(P, ss, G::SEG);
      const bool any = !(P.opts & XYWS_OPT_NO_STORE);
      const bool work = !(P.opts & XYWS_OPT_LATX_NOWORK);
      uint32_t edge = 0;
      u32x4 dprev = {0u, 0u, 0u, 0u};
#pragma unroll
      for (uint32_t k = 0; k < IO::K; k++) {
        const bool ok = IO::valid(wave, k);
        const uint32_t a = (ok ? IO::row(wave, k) : 0u) * 1024u + lane * 16u;
        u32x4 d = *reinterpret_cast<const u32x4*>(&L.seg[a]);
        uint32_t idx = 0;
        if (a >= xka) {
          const uint32_t dd = a - xka;
          uint32_t qq = (uint32_t)((float)dd * rF);
          if (qq * F32 > dd) qq--;
          else if ((qq + 1) * F32 <= dd) qq++;
          idx = 1 + qq;
        }
        if (work && idx < nent) d = d ^ lat_mask(L.tab, nent, idx, a);
        const bool whole = ok && a >= lo_r && a + 16u <= hi_r && a + 16u <= stop;
        if (ok && !whole && a < stop && a < hi_r && a + 16u > lo_r) {
          edge |= 1u << k;
          *reinterpret_cast<u32x4*>(&L.seg[a]) = d;  // (stored bytewise below)
        }
        __builtin_amdgcn_raw_buffer_store_b128(d, rs, (whole && any) ? lane * 16u : OOB, IO::row(wave, k) * 1024u,
                                               AUX_ST_STREAM);
        // (the store's data registers stay live past the next store)
        asm volatile("" ::"v"(dprev.x), "v"(dprev.y), "v"(dprev.z), "v"(dprev.w));
        dprev = d;
      }
      asm volatile("s_nop 1" ::"v"(dprev.x), "v"(dprev.y), "v"(dprev.z), "v"(dprev.w));
      // chunks at the batch edges or at the failing point: their in-range
      // bytes (XORed in LDS above; bytes at or past the failing point got a
      // zero mask)
#pragma nounroll
      while (edge && any) {
        const uint32_t k = __builtin_ctz(edge);
        edge &= edge - 1;
        const uint32_t a = IO::row(wave, k) * 1024u + lane * 16u;
#pragma nounroll
        for (uint32_t y = a; y < a + 16u; y++)
          if (y >= lo_r && y < hi_r && y < stop) P.base[ss + y] = L.seg[y];
      }
      // descriptors of the segment's frames below the failing point (their
      // headers from LDS: never XORed)
      if (P.frames && stop && kst > ka) {
        const uint32_t nd = (uint32_t)(kst - ka < nl ? kst - ka : nl);
        for (uint32_t i = dl; i < nd; i += NDL) {
          const uint64_t k = ka + i;
          const uint64_t ord = L.c0 + k;
          if (ord >= P.cap) break;
          const uint64_t x = X0 + k * F;
          const hdr_info h = lat_hdr(P, L.seg, (uint32_t)(x - ss), x);
          if (h.hlen) write_frame(P, ord, x, h, x + h.hlen, 0);
        }
      }
    }
    it++;
    // the control wave raises the decided prefix while the data waves store
    if (clk.on && cl) clk.acc[LT_SEGS - 16]++;
    cur = nxt;
  }
  clk.mark(cl ? LT_C_ADV : LT_D_ST);
  clk.flush(P);
  if (DT && tid == IO::CLAIM) L.nsl = nsl;  // (lat_check's list length)
}

// Speculative stores (lat_loop): a workgroup's list of the segments it stored
// before every earlier one had decided, and the lattice index each segment's
// stores stop at, goes to its slice of P.lsl when its work ends (n, then
// {segment, index} pairs; LAT_LSW words per workgroup).
constexpr uint32_t LAT_LSW = 1 + 2 * LAT_SLIST;
template <class G, class LL>
XYWS_DEV void lat_dump_list(const run_params& P, const LL& L, uint32_t tid) {
  const uint32_t n = L.nsl;
  uint64_t* q = P.lsl + (uint64_t)blockIdx.x * LAT_LSW;
  if (tid == 0) q[0] = n;
  for (uint32_t i = tid; i < n; i += G::NT) {
    q[1 + 2 * i] = L.sl_seg[i];
    q[2 + 2 * i] = L.sl_k[i];
  }
}

// The undo of segment s's stores past the final failing point kb (whole
// workgroup; the finisher, every workgroup done): the stores reached lattice
// index kst > kb (the segment stored before the failing point was
// published); the bytes from X0 + kb*F to where they stopped get the same
// masks again (XOR is an involution), each frame's key from its header in
// memory (headers are never written by a decode). Rare: a lattice broken in
// the middle of a batch, after the first segments.
template <class G, class LL>
XYWS_DEV void lat_undo(const run_params& P, const LL& L, uint32_t tid, uint64_t s, uint64_t kst, uint64_t kb) {
  const uint64_t X0 = L.X0, F = L.F, kmax = L.kmax;
  const uint64_t ss = s * G::SEG;
  const uint32_t stop = (uint32_t)(X0 + kst * F - ss < G::SEG ? X0 + kst * F - ss : G::SEG);
  const uint32_t lo_r = lat_rel(P.lo, ss), hi_r = P.hi - ss < G::SEG ? (uint32_t)(P.hi - ss) : G::SEG;
  const uint32_t top = stop < hi_r ? stop : hi_r;
  const uint32_t from = lat_rel(X0 + kb * F, ss);  // (the run decoder's bytes: decoded again from there)
  for (uint32_t a = (from & ~15u) + tid * 16u; a < top; a += G::NT * 16u) {
    // the chunk's frames: g (at or before a) and g + 1, below kst
    uint64_t g = a + ss < X0 ? NONE : (a + ss - X0) / F;  // (NONE: the carried frame)
    u32x4 m = {0u, 0u, 0u, 0u};
    for (int t = 0; t < 2; t++, g = g == NONE ? 0 : g + 1) {
      uint4 en = {0u, 0u, 0u, 0u};
      if (g == NONE) {
        const cstate S0 = L.S0;
        if (!(S0.st & S_NOCOV)) en = uint4{lat_rel(S0.cov_ps, ss), lat_rel(X0, ss), S0.cov_kw, 0u};
      } else if (g < kst && g < kmax) {
        const uint64_t x = X0 + g * F;
        const hdr_info h = hdr_global(P, x, NONE);
        if (h.hlen) {
          const uint64_t ps = x + h.hlen;
          const uint64_t end = g + 1 == kmax ? sat_add(ps, h.plen) : x + F;
          en = uint4{lat_rel(ps, ss), lat_rel(end < P.hi ? end : P.hi, ss), aligned_key(h.key, ps, 0), 0u};
        }
      }
      m |= span_key16(a, en.x, en.y, en.z);
    }
    if (a >= from && a >= lo_r && a + 16u <= top) {
      // a whole chunk: four dwords (agent scope: past this CU's caches, which
      // may hold the bytes as loaded); bytes under a zero mask (headers) are
      // written back unchanged (no other writer runs: the run decoder comes
      // after this kernel in the stream)
      uint32_t* q = reinterpret_cast<uint32_t*>(P.base + ss + a);
      const uint32_t mm[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        if (!mm[i]) continue;
        const uint32_t v = __hip_atomic_load(q + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q + i, v ^ mm[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      continue;
    }
#pragma unroll
    for (uint32_t b = 0; b < 16; b++) {
      const uint32_t y = a + b;
      const uint32_t mw = b < 4 ? m.x : b < 8 ? m.y : b < 12 ? m.z : m.w;
      const uint8_t kbyte = (uint8_t)(mw >> (8u * (b & 3u)));
      if (kbyte && y >= from && y >= lo_r && y < top) {
        uint8_t* q = P.base + ss + y;
        const uint8_t v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q, (uint8_t)(v ^ kbyte), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Polls of LW_LOOPS before a workgroup that knew of a failing point gives up
// undoing its own stores and leaves its list to the finisher (every loop has
// ended by the finisher's time, LW_BRK is final there): a wait bounded well
// below anything a stalled grid could cost, and never an undo with a failing
// point that may still move (workgroups of this grid may not be resident yet,
// e.g. while a kernel on another stream holds CUs).
constexpr uint32_t LAT_UNDO_POLLS = 2048;

// Everything after the prologue, for the geometry it chose (every workgroup
// the same: the choice is a function of the batch's first frame): the
// segment loop, the end-of-work undo, the done count and the finisher.
template <class G, class LL>
XYWS_DEV void lat_body(const run_params& P, LL& L, uint32_t tid, uint32_t ahead) {
  using IO = lat_io<G>;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(P.lat + LW_CNT);
  if (!L.na) {
    if constexpr (IO::CTRL) {
      // (a wave-uniform branch: each loop is a scalar branch target)
      if (__builtin_amdgcn_readfirstlane(tid >> 6) == 0)
        lat_loop<G, LR_CTRL>(P, L, tid, ahead);
      else
        lat_loop<G, LR_DATA>(P, L, tid, ahead);
    } else {
      lat_loop<G, LR_ALL>(P, L, tid, ahead);
    }
    __syncthreads();
    // A failing point known when this workgroup's work ends: once every
    // workgroup's segment loop has ended (LW_BRK final: a segment raises it
    // before it publishes, and no segment is decoded after the loops end; no
    // loop waits for anything here) the workgroup undoes its own speculative
    // stores past it, all workgroups in parallel (a break near the batch start
    // after an ungated first round: up to a segment per workgroup). When the
    // loops have not all ended within LAT_UNDO_POLLS polls, or the failing
    // point was raised later, the list goes to the finisher, which undoes it
    // with the final LW_BRK (dumped lists are emptied here once undone).
    // (L.quit: a failing point this workgroup knew of, its own or LW_BRK as
    // read during its loop: no extra load when none was)
    if (tid < 64) {
      uint64_t b = 0;
      if (tid == 0) __hip_atomic_fetch_add(P.lat + LW_LOOPS, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (L.quit && L.nsl) {
        const uint32_t polls = (P.opts & XYWS_OPT_TEST_LATDUMP) ? 0u : LAT_UNDO_POLLS;
        bool ended = false;
        for (uint32_t it = 0; it < polls; it++) {
          if (uniform64(st_load(P.lat + LW_LOOPS)) >= gridDim.x) {
            ended = true;
            break;
          }
          __builtin_amdgcn_s_sleep(8);
        }
        if (ended) b = uniform64(st_load(P.lat + LW_BRK));
      }
      if (tid == 0) L.kbf = b && L.nsl ? ~b : NONE;
    }
    __syncthreads();
    const uint64_t kb = L.kbf;
    if (kb != NONE) {
      const uint32_t n = L.nsl;
      for (uint32_t j = 0; j < n; j++)
        if (kb < L.sl_k[j]) lat_undo<G>(P, L, tid, L.sl_seg[j], L.sl_k[j], kb);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) L.nsl = 0;
      __syncthreads();
    }
    lat_dump_list<G>(P, L, tid);
  }
  // end of the workgroup: the last one to finish writes the call's outputs
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t last = atomicAdd(cnt + 1, 1u) + 1 == gridDim.x ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    L.done_last = last;
  }
  __syncthreads();
  if (!L.done_last) return;
  // the last workgroup: every segment has decided, LW_BRK is final; stores
  // past it are undone (every workgroup's list)
  if (tid == 0) {
    const uint64_t b = st_load(P.lat + LW_BRK);
    L.kbf = b && !L.na ? ~b : NONE;
  }
  __syncthreads();
  const uint64_t kb = L.kbf;
  if (kb != NONE) {
    // the stores to undo, from every workgroup's list at once (one thread per
    // list) into this workgroup's own list in LDS; more than it holds: one
    // list at a time (rare twice over)
    if (tid == 0) L.nsl = 0;
    __syncthreads();
    for (uint32_t w = tid; w < gridDim.x; w += G::NT) {
      const uint64_t* q = P.lsl + (uint64_t)w * LAT_LSW;
      const uint32_t n = (uint32_t)st_load(q);
      for (uint32_t i = 0; i < n; i++) {
        const uint64_t kst = st_load(q + 2 + 2 * i);
        if (kb < kst) {
          const uint32_t j = atomicAdd(&L.nsl, 1u);
          if (j < LAT_SLIST) {
            L.sl_seg[j] = st_load(q + 1 + 2 * i);
            L.sl_k[j] = kst;
          }
        }
      }
    }
    __syncthreads();
    const uint32_t nu = L.nsl;
    if (nu <= LAT_SLIST) {
      for (uint32_t j = 0; j < nu; j++) lat_undo<G>(P, L, tid, L.sl_seg[j], L.sl_k[j], kb);
    } else {
      for (uint32_t w = 0; w < gridDim.x; w++) {
        const uint64_t* q = P.lsl + (uint64_t)w * LAT_LSW;
        const uint32_t n = (uint32_t)st_load(q);
        for (uint32_t i = 0; i < n; i++) {
          const uint64_t kst = st_load(q + 2 + 2 * i);
          if (kb < kst) lat_undo<G>(P, L, tid, st_load(q + 1 + 2 * i), kst, kb);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // (the group counters back to zero for the next call)
  for (uint64_t g = tid; g * LAT_GRP < P.nseg; g += G::NT)
    __hip_atomic_store(P.lgrp + g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid < LAT_NREP) __hip_atomic_store(P.lbrk + LAT_REPW * tid, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid != 0) return;
  lat_finish(P, L);
}

// The kernel: GA's loop for batches whose first frame is at least
// LAT5_MIN_FRAME bytes, GB's otherwise (GA == GB: one loop, the test
// geometry). The segment count is the chosen geometry's (P.nseg from the host
// is unused; the grid covers the smaller segments, workgroups past the
// segment count exit after their done count).
template <class GA, class GB>
__global__ void __launch_bounds__(GB::NT)
__attribute__((amdgpu_waves_per_eu(GB::NT >= 256 ? GB::NT / 256 : 1))) k_stream_lattice(run_params P0) {
  using GL = llay<GA, GB>;
  using IO = lat_io<GB>;
  static_assert(lat_io<GA>::CLAIM == IO::CLAIM, "one claim lane");
  extern __shared__ __attribute__((aligned(256))) uint8_t xs_lds[];
  lat_lds<GL>& L = *reinterpret_cast<lat_lds<GL>*>(xs_lds);
  const uint32_t tid = threadIdx.x;
  uint32_t ahead = NONE32;  // claim lane: the segment claimed one iteration ahead
  // (the prologue: the control lane's dependent round trips — {the epoch and
  // the device policy word, the carry, the first header at the batch start},
  // then two lattice points; a carried frame adds one for the first header.
  // Issuing the static first segment's rows before it measured no faster: c1
  // 0.1110 vs 0.1102 ms, c2 0.1245 vs 0.1246, same box, r05d)
  if (tid == 0) {
    // One round trip for the granule {device policy word, epoch}, the carry
    // and the dwords at the batch start (the first frame's header when
    // nothing is carried: the usual case), all issued before one wait.
    const xyws_carry* cz = P0.cin_user ? P0.cin_user : &k_zero_carry;
    carry_words cc;
    uint32_t r0[5];
    uint64_t dp, ep;
    {
      // (the granule first, inline asm without a wait: the compiler neither
      // waits for it nor moves the plain loads before it; one wait for all)
      u32x4 g;
      asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(g) : "v"(P0.lat + LW_DPOL) : "memory");
#pragma unroll
      for (int i = 0; i < 8; i++) cc.w[i] = reinterpret_cast<const uint64_t*>(cz)[i];
      // (unconditional loads, addresses clamped to the batch's last dword:
      // a branch per dword made the compiler wait after each)
      const uint64_t a0 = P0.lo & ~3ull, dl = (P0.hi + 3) & ~3ull;
#pragma unroll
      for (int i = 0; i < 5; i++) {
        const uint64_t q = a0 + 4 * i;
        r0[i] = *reinterpret_cast<const uint32_t*>(P0.base + (q < dl ? q : dl - 4));
      }
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(g)::"memory");
#pragma unroll
      for (int i = 0; i < 5; i++)
        if (a0 + 4 * i >= dl) r0[i] = 0u;
      dp = (uint64_t)g.x | ((uint64_t)g.y << 32);
      ep = (uint64_t)g.z | ((uint64_t)g.w << 32);
    }
    L.E = ep + 1;
    // the previous call in this stream (LW_DPOL, its finisher's): after an
    // irregular one the run decoder takes this batch whole at once (unless
    // the caller forces the lattice), after one the lattice decoder finished
    // the first segments are not gated
    const bool dvalid = dp >> 63, dreg = (dp & ((1ull << 48) - 1)) >= LAT_FMIN;
    const uint64_t ddec = (dp >> 48) & 0x7Fu;
    uint32_t na = dvalid && !dreg && !(P0.opts & XYWS_OPT_LATTICE) ? 2u : 0u;
    L.nogate = dvalid && dreg && ddec == DEC_LATTICE && !(P0.opts & XYWS_OPT_LAT_GATE) ? 1u : 0u;
    uint64_t c0 = 0;
    const cstate S0 = initial_state_w(P0, cc, c0);
    if (!na && ((S0.st & S_PARTIAL) || S0.X >= P0.hi)) na = 1u;
    uint64_t F = 0, kmax = 0;
    if (!na) {
      hdr_info h;
      if (S0.X == P0.lo) {
        const uint32_t sh = (uint32_t)(P0.lo & 3);
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(r0[i + 1], r0[i], sh);
        const uint64_t room = P0.hi - P0.lo;
        h = parse_header_words(w, room < 16 ? (uint32_t)room : 16u);
      } else {
        h = hdr_global(P0, S0.X, NONE);
      }
      F = sat_add(h.hlen, h.plen);
      if (!h.hlen || F < LAT_FMIN || F > LAT_FMAX) na = 1;
      else kmax = (P0.hi - S0.X + F - 1) / F;
    }
    // Lattice points 1 and 2 (X0 + F, X0 + 2F) from memory before anything is
    // stored: a batch whose frames change size there (an irregular batch after
    // regular ones) goes to the run decoder whole at once, at the cost of this
    // workgroup's first rows (not a gated first round of every workgroup).
    // (Not in the blind test mode, whose breaks at frame 1 exercise the undo.)
    if (!na && kmax > 1 && !(P0.opts & (XYWS_OPT_TEST_LATSPEC | XYWS_OPT_LATX_NOCHK))) {
      const uint64_t dl = (P0.hi + 3) & ~3ull;
      uint32_t r[2][5];
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const uint64_t a = (S0.X + (j + 1) * F) & ~3ull;
#pragma unroll
        for (int i = 0; i < 5; i++) {
          const uint64_t q = a + 4 * i;
          r[j][i] = (j == 0 || kmax > 2) && q < dl ? *reinterpret_cast<const uint32_t*>(P0.base + q) : 0u;
        }
      }
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const uint64_t k = j + 1;
        if (k >= kmax) break;
        const uint64_t x = S0.X + k * F;
        const uint32_t sh = (uint32_t)(x & 3);
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(r[j][i + 1], r[j][i], sh);
        const uint64_t room = P0.hi - x;
        const hdr_info h = parse_header_words(w, room < 16 ? (uint32_t)room : 16u);
        const bool last = k + 1 == kmax;
        const uint64_t fend = h.hlen ? sat_add(x + h.hlen, h.plen) : x;
        const bool ok = h.hlen ? ((uint64_t)h.hlen + h.plen == F && h.plen < F) || (last && fend >= P0.hi) : last;
        if (!ok) na = 1;
      }
    }
    // the loop's geometry: GA's segments for large frames
    const bool big = GA::SEG != GB::SEG && !na && F >= LAT5_MIN_FRAME;
    const uint64_t seg = big ? GA::SEG : GB::SEG;
    const uint64_t nseg = (P0.hi + seg - 1) / seg;
    L.nseg = nseg;
    L.S0 = S0;
    L.c0 = c0;
    L.X0 = S0.X;
    L.F = F;
    L.kmax = kmax;
    L.na = na;
    L.quit = 0;
    L.nsl = 0;
    L.big = big ? 1u : 0u;
    // the first round is static (segment b, then b + grid: every workgroup's
    // first segment, the one its gate holds, is among the first grid
    // segments, so no gate waits on a segment that waits itself), then claims
    // from the counter offset by 2 * grid (lat_loop)
    L.cur = !na && blockIdx.x < nseg ? blockIdx.x : NONE32;
  }
  if (tid == IO::CLAIM) ahead = blockIdx.x - gridDim.x;  // (+ 2 * grid at its use: b + grid)
  __syncthreads();
  run_params P = P0;
  P.nseg = uniform64(L.nseg);
  P.opts &= ~XYWS_OPT_LAT_NOGATE;
  if (uniform32(L.nogate)) P.opts |= XYWS_OPT_LAT_NOGATE;
  if constexpr (GA::SEG != GB::SEG) {
    if (uniform32(L.big)) {
      lat_body<GA>(P, L, tid, ahead);
      return;
    }
  }
  lat_body<GB>(P, L, tid, ahead);
}
