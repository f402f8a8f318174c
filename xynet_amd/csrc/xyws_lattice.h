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
//  * Segments of SEG bytes are claimed in batch order from one counter, one
//    claim ahead (the next segment's loads fly while the current one is
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
//    segment publishes its own result (AGG: its points hold; BRK: one failed),
//    then looks back over the published results of the segments before it
//    (decoupled look-back, 64 per round; a segment that saw its prefix hold
//    publishes INCL, which ends later look-backs) and stores only when every
//    earlier point held: nothing is ever stored speculatively, so nothing is
//    ever undone.
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
  LW_EPOCH = 1,    // completed calls (a call runs with E = this + 1)
  LW_BRK = 2,      // ~(earliest failing lattice index) of this call, 0 = none (reset by the finisher)
  LW_UNMASK = 3,   // xyws_unmask's claim counter pair (u32 claims, u32 done; reset by its last workgroup)
  LW_REDIR = 8,    // redirect record for the run decoder: [0] state, [1] p, [2] frames before p
  LW_RCARRY = 16,  // the carry the run decoder starts from at p (8 words)
  LW_STAT = 32     // per segment: (E << 2) | LS_*
};
enum { LS_AGG = 1, LS_INCL = 2, LS_BRK = 3 };
enum : uint64_t { RD_DONE = 0, RD_FULL = 1, RD_FROM = 2 };

template <uint32_t NT_, uint32_t SEG_>
struct lgeom {
  static constexpr uint32_t NT = NT_, SEG = SEG_, CH = SEG_ / 16 / NT_;
  static constexpr uint32_t TMAX = SEG_ / LAT_FMIN + 3;  // covering frame + lattice points
  static_assert(CH * 16 * NT == SEG, "whole chunks per lane");
};
using G_LAT = lgeom<1024, 131072>;
using G_LAT_SMALL = lgeom<64, 1024>;  // tests: 1 KiB segments, many segment boundaries

template <class G>
struct __attribute__((aligned(16))) lat_lds {
  uint8_t seg[G::SEG + 32];  // the segment and the 16 bytes after it
  uint4 tab[G::TMAX];        // frames overlapping the segment: {ps, end, kw, 0} segment-relative
  cstate S0;                 // the state at the batch start (carry)
  uint64_t E, X0, F, kmax, c0, brk_g;
  uint32_t na, cur, nxt, brk, go, quit, done_last;
};

// Segment-relative clamp of an absolute position to [0, 2^32).
XYWS_DEV uint32_t lat_rel(uint64_t x, uint64_t ss) {
  if (x <= ss) return 0;
  const uint64_t d = x - ss;
  return d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
}

// The decoupled look-back of segment s (wave 0, every lane; the result in
// every lane): 1 when every lattice point before segment s held (an INCL
// among the predecessors with only AGG between), 0 when one failed (a BRK, or
// a failing index before the segment in LW_BRK). Segments are claimed only by
// running workgroups and a segment's result depends on nothing but its own
// bytes, so every wait ends; the bound reports a bug (device error bit 2).
XYWS_DEV int lat_lookback(const run_params& P, uint64_t s, uint64_t E, uint64_t k_first, uint32_t lane) {
  if (s == 0) return 1;
  const uint64_t* stat = P.lat + LW_STAT;
  uint64_t j = s;
  for (uint32_t it = 0; it < (1u << 22); it++) {
    const uint64_t b = st_load(P.lat + LW_BRK);
    if (b && ~b < k_first) return 0;  // a point before this segment failed
    const bool valid = j >= 1 + (uint64_t)lane;
    const uint64_t v = valid ? st_load(stat + (j - 1 - lane)) : ((E << 2) | LS_INCL);
    const bool pub = (v >> 2) == E;
    const uint32_t st = (uint32_t)v & 3u;
    const uint64_t stop = __ballot(!pub || st >= LS_INCL);
    if (!stop) {
      j -= 64;  // 64 predecessors whose own points held: further back
      continue;
    }
    const uint32_t f = (uint32_t)__builtin_ctzll(stop);
    const uint64_t vf = shfl64(v, f);
    if ((vf >> 2) != E) {  // the nearest undecided predecessor: wait for it
      __builtin_amdgcn_s_sleep(1);
      j = s;
      continue;
    }
    return ((uint32_t)vf & 3u) == LS_INCL ? 1 : 0;
  }
  if (lane == 0) atomicOr(P.head + 1, 2u);
  return 0;
}

// XOR mask of the 16-byte chunk at segment offset a from the table: entry
// `idx` and the one after it (a chunk meets at most two frames, F >= 16).
XYWS_DEV u32x4 lat_mask(const uint4* tab, uint32_t nent, uint32_t idx, uint32_t a) {
  const uint4 g = tab[idx];
  if (g.x <= a && a + 16u <= g.y) return u32x4{g.z, g.z, g.z, g.z};
  u32x4 m;
  m.x = g.z & range_mask32(a, g.x, g.y);
  m.y = g.z & range_mask32(a + 4, g.x, g.y);
  m.z = g.z & range_mask32(a + 8, g.x, g.y);
  m.w = g.z & range_mask32(a + 12, g.x, g.y);
  if (idx + 1 < nent) {
    const uint4 n = tab[idx + 1];
    if (n.x < a + 16u) {
      m.x |= n.z & range_mask32(a, n.x, n.y);
      m.y |= n.z & range_mask32(a + 4, n.x, n.y);
      m.z |= n.z & range_mask32(a + 8, n.x, n.y);
      m.w |= n.z & range_mask32(a + 12, n.x, n.y);
    }
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
template <class G>
XYWS_DEV void lat_finish(const run_params& P, lat_lds<G>& L) {
  uint64_t* rd = P.lat + LW_REDIR;
  const xyws_carry* cz = P.cin_user ? P.cin_user : &k_zero_carry;
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
      if (P.pol) {
        const uint64_t v[5] = {L.E, P.hi - P.lo, F, F, 3};
#pragma unroll
        for (int i = 1; i < 5; i++) __hip_atomic_store(P.pol + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(P.pol, v[0], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      st_store(rd, RD_DONE);
    }
  }
  uint32_t* cnt = reinterpret_cast<uint32_t*>(P.lat + LW_CNT);
  st_store(P.lat + LW_BRK, 0);
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

template <class G>
__global__ void __launch_bounds__(G::NT, 1) k_stream_lattice(run_params P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t xs_lds[];
  lat_lds<G>& L = *reinterpret_cast<lat_lds<G>*>(xs_lds);
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(P.lat + LW_CNT);
  uint32_t ahead = NONE32;  // lane 0: the segment claimed one iteration ahead
  if (tid == 0) {
    L.E = st_load(P.lat + LW_EPOCH) + 1;
    const xyws_carry* cz = P.cin_user ? P.cin_user : &k_zero_carry;
    uint64_t c0 = 0;
    const cstate S0 = initial_state(P, cz, c0);
    uint32_t na = (S0.st & S_PARTIAL) || S0.X >= P.hi ? 1u : 0u;
    uint64_t F = 0, kmax = 0;
    if (!na) {
      const hdr_info h = hdr_global(P, S0.X, NONE);
      F = sat_add(h.hlen, h.plen);
      if (!h.hlen || F < LAT_FMIN || F > LAT_FMAX) na = 1;
      else kmax = (P.hi - S0.X + F - 1) / F;
    }
    L.S0 = S0;
    L.c0 = c0;
    L.X0 = S0.X;
    L.F = F;
    L.kmax = kmax;
    L.na = na;
    L.quit = 0;
    L.cur = NONE32;
    if (!na) {
      const uint32_t c = atomicAdd(cnt, 1u);
      if (c < P.nseg) {
        L.cur = c;
        const uint32_t a = atomicAdd(cnt, 1u);
        ahead = a < P.nseg ? a : NONE32;
      }
    }
  }
  __syncthreads();
  const uint64_t E = uniform64(L.E);
  if (!L.na) {
    const uint64_t X0 = uniform64(L.X0), F = uniform64(L.F), kmax = uniform64(L.kmax);
    const float rF = 1.0f / (float)(F < (1ull << 24) ? F : (1ull << 24));
    const uint32_t F32 = F < 0x80000000ull ? (uint32_t)F : 0x80000000u;
    uint32_t cur = uniform32(L.cur);
    u32x4 e[G::CH];
    u32x4 epad = {0u, 0u, 0u, 0u};
    auto issue = [&](uint32_t s) {
      const __amdgpu_buffer_rsrc_t rs = lat_rsrc(P, (uint64_t)s * G::SEG, G::SEG + 16);
#pragma unroll
      for (uint32_t k = 0; k < G::CH; k++)
        e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16u, k * G::NT * 16u, AUX_NT);
      if (tid == 0) epad = __builtin_amdgcn_raw_buffer_load_b128(rs, 0u, G::SEG, AUX_NT);
    };
    if (cur != NONE32) issue(cur);
    while (cur != NONE32) {
      uint32_t t = tid;
      asm volatile("" : "+v"(t));  // (lane address math per segment: see sweep_loop)
      const uint64_t ss = (uint64_t)cur * G::SEG;
      __syncthreads();  // the previous segment's LDS reads are done
#pragma unroll
      for (uint32_t k = 0; k < G::CH; k++) *reinterpret_cast<u32x4*>(&L.seg[(k * G::NT + t) * 16u]) = e[k];
      if (t == 0) {
        *reinterpret_cast<u32x4*>(&L.seg[G::SEG]) = epad;
        L.nxt = ahead;
        if (ahead != NONE32) {
          if (L.quit) {
            ahead = NONE32;
          } else {
            const uint32_t a = atomicAdd(cnt, 1u);
            ahead = a < P.nseg ? a : NONE32;
          }
        }
        L.brk = NONE32;
      }
      __syncthreads();
      const uint32_t nxt = uniform32(L.nxt);
      if (nxt != NONE32) issue(nxt);  // (in flight through the checks, the look-back and the stores)
      // lattice points in the segment: k in [ka, kz)
      const uint64_t se = ss + G::SEG;
      const uint64_t ka = ss <= X0 ? 0 : (ss - X0 + F - 1) / F;
      uint64_t kz = se <= X0 ? 0 : (se - X0 + F - 1) / F;
      if (kz > kmax) kz = kmax;
      const uint32_t nl = kz > ka ? (uint32_t)(kz - ka) : 0u;
      const uint32_t xka = ka < kmax ? lat_rel(X0 + ka * F, ss) : 0xFFFFFFFFu;  // first lattice point (relative)
      // entry 0: the frame covering the segment's first bytes
      if (t == G::NT - 1) {
        uint4 c = {0u, 0u, 0u, 0u};
        if (ka == 0) {
          const cstate S0 = L.S0;
          if (!(S0.st & S_NOCOV)) c = uint4{lat_rel(S0.cov_ps, ss), lat_rel(X0, ss), S0.cov_kw, 0u};
        } else {
          const uint64_t xc = X0 + (ka - 1) * F;
          const hdr_info h = hdr_global(P, xc, NONE);
          if (h.hlen) {
            const uint64_t ps = xc + h.hlen;
            const uint64_t end = ka - 1 + 1 == kmax ? sat_add(ps, h.plen) : xc + F;
            c = uint4{lat_rel(ps, ss), lat_rel(end < P.hi ? end : P.hi, ss), aligned_key(h.key, ps, 0), 0u};
          }
        }
        L.tab[0] = c;
      }
      // entries 1..nl: the lattice points, each checked by one lane
      for (uint32_t i = t; i < nl; i += G::NT) {
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
      __syncthreads();
      const uint32_t brk = uniform32(L.brk);
      if (t == 0) {
        if (brk != NONE32)
          __hip_atomic_fetch_max(P.lat + LW_BRK, ~(ka + brk), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st_store(P.lat + LW_STAT + cur, (E << 2) | (brk != NONE32 ? LS_BRK : LS_AGG));
      }
      if (t < 64) {
        const int go = lat_lookback(P, cur, E, ka, lane);
        if (t == 0) {
          L.go = (uint32_t)go;
          if (go && brk == NONE32) st_store(P.lat + LW_STAT + cur, (E << 2) | LS_INCL);
          if (!go || brk != NONE32) L.quit = 1;  // the rest of the batch is the run decoder's
        }
      }
      __syncthreads();
      // stores: every chunk below the first failing point (nothing when an
      // earlier point failed); entries past it are left out
      const uint32_t go = uniform32(L.go);
      const uint32_t nent = brk != NONE32 ? 1u + brk : 1u + nl;
      const uint32_t stop = !go ? 0u : brk != NONE32 ? (uint32_t)(X0 + (ka + brk) * F - ss) : G::SEG;
      const uint32_t lo_r = lat_rel(P.lo, ss), hi_r = P.hi - ss < G::SEG ? (uint32_t)(P.hi - ss) : G::SEG;
      const __amdgpu_buffer_rsrc_t rs = lat_rsrc(P, ss, G::SEG);
      const bool any = !(P.opts & XYWS_OPT_NO_STORE);
      u32x4 dprev = {0u, 0u, 0u, 0u};
      uint32_t edge = 0;
#pragma unroll
      for (uint32_t k = 0; k < G::CH; k++) {
        const uint32_t a = (k * G::NT + t) * 16u;
        uint32_t idx = 0;
        if (a >= xka) {
          const uint32_t d = a - xka;
          uint32_t qq = (uint32_t)((float)d * rF);
          if (qq * F32 > d) qq--;
          else if ((qq + 1) * F32 <= d) qq++;
          idx = 1 + qq;
        }
        const u32x4 v = *reinterpret_cast<const u32x4*>(&L.seg[a]);
        const u32x4 m = idx < nent ? lat_mask(L.tab, nent, idx, a) : u32x4{0u, 0u, 0u, 0u};
        const bool whole = a >= lo_r && a + 16u <= hi_r && a + 16u <= stop;
        if (!whole && a < stop && a < hi_r && a + 16u > lo_r) edge |= 1u << k;
        const u32x4 d = v ^ m;
        __builtin_amdgcn_raw_buffer_store_b128(d, rs, (whole && any) ? t * 16u : OOB, k * G::NT * 16u, AUX_ST);
        asm volatile("" ::"v"(dprev.x), "v"(dprev.y), "v"(dprev.z), "v"(dprev.w));
        dprev = d;
      }
      asm volatile("s_nop 1" ::"v"(dprev.x), "v"(dprev.y), "v"(dprev.z), "v"(dprev.w));
      // chunks at the batch edges or at the failing point: their in-range bytes
#pragma nounroll
      while (edge && any) {
        const uint32_t k = __builtin_ctz(edge);
        edge &= edge - 1;
        const uint32_t a = (k * G::NT + t) * 16u;
        uint32_t idx = 0;
        if (a >= xka) idx = 1 + (a - xka) / F32;
        if (idx >= nent) continue;
        const u32x4 m = lat_mask(L.tab, nent, idx, a);
#pragma nounroll
        for (uint32_t b = 0; b < 16; b++) {
          const uint32_t y = a + b;
          const uint32_t mw = b < 4 ? m.x : b < 8 ? m.y : b < 12 ? m.z : m.w;
          const uint8_t kb = (uint8_t)(mw >> (8u * (b & 3u)));
          if (kb && y >= lo_r && y < hi_r && y < stop) P.base[ss + y] = L.seg[y] ^ kb;
        }
      }
      // descriptors of the segment's frames below the failing point
      if (P.frames && go) {
        const uint32_t nd = brk != NONE32 ? brk : nl;
        for (uint32_t i = t; i < nd; i += G::NT) {
          const uint64_t k = ka + i;
          const uint64_t ord = L.c0 + k;
          if (ord >= P.cap) break;
          const uint64_t x = X0 + k * F;
          const hdr_info h = lat_hdr(P, L.seg, (uint32_t)(x - ss), x);
          if (h.hlen) write_frame(P, ord, x, h, x + h.hlen, 0);
        }
      }
      cur = nxt;
    }
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
  if (!L.done_last || tid != 0) return;
  lat_finish<G>(P, L);
}
