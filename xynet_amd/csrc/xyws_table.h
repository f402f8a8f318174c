// xyws_table.h — the table decoder of xyws_decode_stream for irregular batches
// (frames of mixed sizes, mostly large: SURVEY §8(d) config 4), included by
// xyws_stream.hip after xyws_lattice.h (it shares run_params, the header
// readers, the run decoder's entry scan, the lattice decoder's redirect record
// and its store helpers).
//
// The frame chain of a batch is a linked list (websocket_frame_header.h:305-385:
// frame k+1 starts at start_k + H_k + P_k). The run decoder walks it while it
// streams, one fixed byte range per CU, and pays for that: a range's length is
// fixed while the frames in it are not (the CUs finish over a 50-100 us spread),
// the chase sits between a segment's loads and its stores, and the register
// budget of one loop holding both spills. This decoder separates the two:
//
//  1. k_stream_index (the index): one workgroup per run range (whole
//     segments). Run 0 starts at the batch's first frame (exact: the batch
//     start and the carry); every other run finds its entry with the run
//     decoder's scan (find_entry: the earliest position of its range whose
//     chain of 2/6/8 headers is plausible for a client stream) and walks the
//     headers only, from a 1 KiB window per hop, up to the first frame start
//     at or after its range end (its exit). It records every frame (an
//     xyws_frame, the descriptor the caller may ask for) and writes, per
//     segment, a 256-byte descriptor: how many frames start in it and the
//     first TD_K of them as segment-relative {payload start, payload end, key
//     word} entries, and the frame covering its first byte (slot A: a frame of
//     the same run; slot B: written by the run whose frame crosses into this
//     range). The workgroup that finishes last checks the hand-overs: run r's
//     entry must be where the chain from run 0 arrives (the exit of the
//     nearest earlier run with an entry), or, for a run without one, the
//     chain must jump past its range. By induction from run 0 every run
//     before the first mismatch is exact; the batch up to that run's expected
//     entry p is covered. It writes the call's outputs (count, carry, the
//     decoder-choice words) when everything is covered, or the lattice
//     decoder's redirect record (RD_FROM p: the run decoder takes the rest,
//     frame count and ordinals continued).
//  2. k_stream_table (the stream): the lattice decoder's streaming loop
//     (claimed 128 KiB segments staged in LDS, the next segment's rows in
//     registers, one 16-byte nontemporal store per chunk) with the segment's
//     frame table loaded from its descriptor (by the claim wave, one segment
//     ahead, with the rows) instead of checked on a lattice. Each chunk is
//     XORed with the keys of the frames it overlaps (websocket_frame_mask.h:
//     6-25 per frame, from phase 0); header bytes are never written.
//  3. k_table_emit: the descriptors (only when the caller asks), one
//     workgroup per run, copied from the records at their ordinals.
//
// Any byte stream decodes exactly as the reference parses it: a wrong entry
// (payload bytes that look like a header chain), a run whose frames do not fit
// its record list or a segment whose frames do not fit the stream kernel's
// table only move the point from which the run decoder takes over.

// The stream kernel's geometry: NT threads, SEG-byte segments (whole 1 KiB
// rows, the same number per wave); run ranges are whole segments.
template <uint32_t NT_, uint32_t SEG_>
struct tgeom {
  static constexpr uint32_t NT = NT_, SEG = SEG_;
  static constexpr uint32_t NMAX = SEG_ / 128 > 8 ? SEG_ / 128 : 8;  // frames starting in one segment (its table)
  static_assert(SEG_ % (1024 * (NT_ / 64)) == 0, "whole rows, the same number per wave");
};
using G_TAB = tgeom<1024, 128 * 1024>;  // 16 waves x 8 rows of 1 KiB
using G_TAB_SMALL = tgeom<64, 1024>;    // tests: 1 KiB segments, many segment boundaries
constexpr uint32_t TD_W = 16;            // 16-byte granules per segment descriptor
constexpr uint32_t TD_K = TD_W - 3;      // frames inline: [0] meta, [1] cover B, [2] cover A, [3..] frames
constexpr uint32_t TSPR_MAX = 2048;      // segments per run range (the index kernel's per-segment counts)
enum : uint32_t { TC_NONE = 0, TC_A = 1, TC_B = 2 };  // meta.z: where the covering frame's entry is
// run record words (TR_WORDS per run)
// (TR_PX: the exit of the run's own chase, {exit, epoch} in one 16-byte
// granule, published as soon as the chase ends: the next run compares its
// entry with it)
// (TR_T0..TR_T2: s_memrealtime at the kernel start, after the entry scan,
// after the chase and its check; TR_T3: the second chase's hops, 0 if none)
enum { TR_H = 0, TR_X = 1, TR_N = 2, TR_OVF = 3, TR_FS = 4, TR_T0 = 5, TR_T1 = 6, TR_T2 = 7, TR_S = 8, TR_T3 = 13,
       TR_PX = 14, TR_WORDS = 16 };
// the table decoder's control words (u64, zeroed at allocation)
enum { TW_DONE = 0,   // u32 [0] index workgroups done, u32 [1] stream workgroups done (reset by the last of each)
       TW_CLAIM = 1,  // u32 [0] the stream kernel's claim counter (reset by its last workgroup)
       TW_RSTAR = 2,  // the first run not covered (R: all)
       TW_PCOV = 3,   // the coverage end p (absolute): bytes from p on are the run decoder's
       TW_EPOCH = 4,  // completed index calls (the decoder-choice words' epoch)
       TW_TAIL = 5,   // [5..7] the frame covering [last exact frame start, p): payload start, end (absolute), key word
       TW_BASE = 64,  // per run: frames before its first true one (ordinal base), 1024 words
       TW_SKIP = 64 + 1024,   // per run: records before its first true frame (a false entry's chain that
                              // joined the true one), 1024 words
       TW_ENT = 64 + 2048,    // per run: its first true frame start (absolute), 1024 words
       TW_WORDS = 64 + 3072 };
constexpr uint64_t TAB_MAX_RUNS = 1024;

struct __attribute__((aligned(16))) idx_ext {
  uint8_t cw[1024 + 32];          // the chase window: 1 KiB at wa, and 16 bytes after it
  uint32_t scnt[TSPR_MAX];        // per own segment: frames starting in it | 1 << 31 when one starts at its first byte
};

// Segment-relative entry {payload start, payload end, key word, 0} of a frame
// whose payload is [ps, pe) (pe already cut at hi) for the segment at ss.
XYWS_DEV uint4 tab_entry(uint64_t ps, uint64_t pe, uint32_t kw, uint64_t ss) {
  return uint4{lat_rel(ps, ss), lat_rel(pe, ss), kw, 0u};
}
XYWS_DEV void st16(uint4* p, const uint4& v) {
  *p = v;
}

template <class G>
struct __attribute__((aligned(16))) idx_lds {
  lds_t<G> L;
  idx_ext X;
};

// The chase of run r (wave 0, every lane the same values): frames from h up
// to the first frame start at or after re. Headers are parsed from a 1 KiB
// window of memory loaded by the wave at the hop (small frames: many hops per
// window). Records, inline segment entries and cover entries are written as
// it goes; returns the exit, the frame count, the final chain state.
template <class G, class TG>
XYWS_DEV void idx_chase(const run_params& P, idx_lds<G>& I, uint32_t lane, uint32_t r, uint64_t h, uint64_t rb,
                        uint64_t re, uint64_t& xout, uint64_t& nout, uint32_t& ovf, cstate& S, uint64_t& fs_last,
                        uint4& last) {
  idx_ext& X = I.X;
  const uint64_t s_own0 = rb / TG::SEG, s_own1 = (re + TG::SEG - 1) / TG::SEG;  // own segments [s_own0, s_own1)
  xyws_frame* list = P.tlist + (uint64_t)r * P.trcap;
  uint64_t x = h, n = 0, wa = NONE;
  ovf = 0;
  fs_last = 0;
  last = uint4{0u, 0u, 0u, 0u};  // the last frame's payload end (absolute, 2 words) and key word
  const uint64_t top = (P.hi + 15) & ~15ull;
  while (x < re && x < P.hi) {
    if (wa == NONE || x < wa || x + XYWS_MAX_FRAME_HEADER_SIZE > wa + 1040) {
      wa = x & ~15ull;
      const uint64_t room = top > wa ? top - wa : 0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          P.base + wa, 0, room < 1040 ? (uint32_t)room : 1040u, 0x00020000);
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16u, 0, 0);
      const u32x4 v2 = __builtin_amdgcn_raw_buffer_load_b128(rs, lane < 1 ? 1024u : OOB, 0, 0);
      *reinterpret_cast<u32x4*>(&X.cw[lane * 16u]) = v;
      if (lane < 1) *reinterpret_cast<u32x4*>(&X.cw[1024]) = v2;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the window's LDS writes before its reads)
    }
    const uint32_t o = (uint32_t)(x - wa), a4 = o & ~3u, sh = o & 3u;
    const uint32_t* q = reinterpret_cast<const uint32_t*>(&X.cw[a4]);
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(q[i + 1], q[i], sh);
    const uint64_t room = P.hi - x;
    const hdr_info hd = parse_header_words(w, room < 16 ? (uint32_t)room : 16u);
    if (!hd.hlen) {  // a header cut by the batch end: the carry
      S.X = x; S.cov_ps = x; S.cov_start = x; S.cov_kw = 0; S.cov_key = 0; S.st = S_PARTIAL | S_NOCOV; S.pad = 0;
      break;
    }
    const uint64_t s = x / TG::SEG;
    const uint32_t k = X.scnt[s - s_own0] & 0x7FFFFFFFu;
    if (n >= P.trcap || k >= TG::NMAX) {  // no room: the run decoder takes the batch from this frame on
      ovf = 1;
      break;
    }
    const uint64_t ps = x + hd.hlen, end = sat_add(ps, hd.plen), pe = end < P.hi ? end : P.hi;
    const uint32_t kw = aligned_key(hd.key, ps, 0);
    if (lane == 0) {
      xyws_frame f;
      f.frame_off = (int64_t)(x - P.lo);
      f.payload_off = (int64_t)(ps - P.lo);
      f.payload_len = hd.plen;
      f.key[0] = (uint8_t)hd.key; f.key[1] = (uint8_t)(hd.key >> 8);
      f.key[2] = (uint8_t)(hd.key >> 16); f.key[3] = (uint8_t)(hd.key >> 24);
      f.flags = hd.flags;
      f.hdr_len = (uint8_t)hd.hlen;
      f.status = (uint8_t)(hd.status | (end > P.hi ? XYWS_ST_PAYLOAD_INCOMPLETE : 0));
      f.reserved = 0;
      list[n] = f;
      if (k < TD_K) st16(P.tdesc + s * TD_W + 3 + k, tab_entry(ps, pe, kw, s * TG::SEG));
    }
    // (every lane writes the same count: each reads back its own write)
    X.scnt[s - s_own0] = (k + 1) | (x == s * TG::SEG ? 0x80000000u : (X.scnt[s - s_own0] & 0x80000000u));
    // the own segments whose first byte this frame covers: (x, pe), each
    // lane one (those of later ranges: from the run's last frame, written
    // once the run's entry has been checked, k_stream_index)
    const uint64_t c1 = x / TG::SEG + 1, c2 = pe ? (pe - 1) / TG::SEG + 1 : 0;  // [c1, c2)
    for (uint64_t c = c1 + lane; c < c2 && c < s_own1; c += 64) {
      const uint64_t ss = c * TG::SEG;
      st16(P.tdesc + c * TD_W + 2, tab_entry(ps, pe, kw, ss));
    }
    last = uint4{(uint32_t)pe, (uint32_t)(pe >> 32), kw, 0u};
    S = frame_state(x, hd);
    fs_last = (uint64_t)hd.hlen + hd.plen;
    n++;
    x = end;
  }
  // own segments past where the chase stopped (a header cut by the batch
  // end): no own frame covers them
  for (uint64_t c = (x < rb ? s_own0 : x / TG::SEG + 1) + lane; c < s_own1; c += 64)
    st16(P.tdesc + c * TD_W + 2, uint4{0u, 0u, 0u, 0u});
  xout = x;
  nout = n;
}

// Index kernel (see the file comment), one workgroup per run range.
template <class G, class TG>
__global__ void __launch_bounds__(G::NT, 1) k_stream_index(run_params P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t xs_lds[];
  idx_lds<G>& I = *reinterpret_cast<idx_lds<G>*>(xs_lds);
  lds_t<G>& L = I.L;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t r = blockIdx.x, R = gridDim.x;
  const uint64_t rb = (uint64_t)r * P.rbytes, re = rb + P.rbytes < P.hi ? rb + P.rbytes : P.hi;
  const uint64_t s_own0 = rb / TG::SEG, s_own1 = (re + TG::SEG - 1) / TG::SEG, nown = s_own1 - s_own0;
  for (uint32_t i = tid; i < nown; i += G::NT) I.X.scnt[i] = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {
    const xyws_carry* cz = P.cin_user ? P.cin_user : &k_zero_carry;
    uint64_t c0 = 0;
    const cstate S0 = initial_state(P, cz, c0);
    L.E = st_load(P.tctl + TW_EPOCH) + 1;
    L.S = S0;
    L.aux2 = c0;
    L.aux0 = NONE;
    L.act = (S0.st & (S_PARTIAL | S_PARTCARRY)) ? 1u : 0u;  // (the run decoder takes such a batch whole)
  }
  __syncthreads();
  const cstate S0 = L.S;
  const bool na = L.act != 0;
  uint64_t h = NONE;
  if (!na) {
    if (r == 0) {
      h = S0.X;
    } else {
      seg_io<G> io;
      find_entry<G>(P, L, io, tid, rb, re);
      h = L.aux0 < re ? L.aux0 : NONE;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  // run 0: the carried frame covers the bytes before X0 (slot A in its own
  // range, B beyond it); a zero entry when nothing is carried
  if (r == 0 && !na) {
    const uint64_t X0 = S0.X;
    const uint64_t c2 = X0 < P.hi ? (X0 + TG::SEG - 1) / TG::SEG : (P.hi + TG::SEG - 1) / TG::SEG;  // segments with ss < X0
    for (uint64_t c = tid; c < c2; c += G::NT) {
      const uint64_t ss = c * TG::SEG;
      uint4 en = {0u, 0u, 0u, 0u};
      if (!(S0.st & S_NOCOV)) en = tab_entry(S0.cov_ps, X0 < P.hi ? X0 : P.hi, S0.cov_kw, ss);
      st16(P.tdesc + c * TD_W + (c < s_own1 ? 2 : 1), en);
    }
  }
  __syncthreads();
  // the chase (wave 0)
  if (tid < 64) {
    const uint64_t E = uniform64(L.E);
    uint64_t x = h, n = 0, fs = 0;
    uint32_t ovf = 0;
    cstate S = S0;
    uint4 last;
    if (h != NONE) idx_chase<G, TG>(P, I, lane, r, h, rb, re, x, n, ovf, S, fs, last);
    uint64_t* rec = P.trec + (uint64_t)r * TR_WORDS;
    if (tid == 0) granule_store(rec + TR_PX, h == NONE ? NONE : x, E);
    // The entry against the chain arriving from before: the own-chase exit
    // of the nearest earlier run with an entry (published as that run's chase
    // ended, without waiting for its own check: no chain of waits). A run
    // whose scan took a false chain (payload bytes that parse as plausible
    // headers) or found nothing while the chain lands in its range chases its
    // range again from there (an exit before the range: an earlier run that
    // stopped short, left to the final check). The workgroup finishing the call checks every
    // hand-over again on the final records (an earlier run's exit that moved
    // with its own second chase).
    if (r >= 1 && !na) {
      uint64_t xp = NONE;
      if (tid == 0) {
        for (int64_t j = (int64_t)r - 1; j >= 0; j--) {
          uint64_t a = 0, b = 0;
          uint32_t it = 0;
          for (;;) {
            granule_load(P.trec + (uint64_t)j * TR_WORDS + TR_PX, a, b);
            if (b == E || ++it >= (1u << 20)) break;
            __builtin_amdgcn_s_sleep(2);
          }
          if (b != E) break;  // (bounded wait timed out: no second chase; the final check decides)
          if (a != NONE) {
            xp = a;
            break;
          }
        }
      }
      xp = uniform64(xp);
      if (xp != NONE && xp >= rb && xp < re && xp != h) {
        for (uint32_t i = lane; i < nown; i += 64) I.X.scnt[i] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        h = xp;
        S = S0;
        idx_chase<G, TG>(P, I, lane, r, h, rb, re, x, n, ovf, S, fs, last);
      }
    }
    // the cover of the segments of later ranges that the run's last frame
    // reaches: only after the check (a false chain's frames never write
    // into another run's descriptors)
    if (n && !ovf) {
      const uint64_t pe = (uint64_t)last.x | ((uint64_t)last.y << 32), ps = S.cov_ps;
      const uint64_t c2 = pe ? (pe - 1) / TG::SEG + 1 : 0;
      for (uint64_t c = s_own1 + lane; c < c2; c += 64)
        st16(P.tdesc + c * TD_W + 1, tab_entry(ps, pe, last.z, c * TG::SEG));
    }
    if (tid == 0) {
      st_store(rec + TR_T0, t0);
      st_store(rec + TR_T1, t1);
      st_store(rec + TR_T2, __builtin_amdgcn_s_memrealtime());
      st_store(rec + TR_H, h);
      st_store(rec + TR_X, h == NONE ? NONE : x);
      st_store(rec + TR_N, n);
      st_store(rec + TR_OVF, ovf);
      st_store(rec + TR_FS, fs);
      put_state(rec + TR_S, S);
      L.cnt = n;
    }
  }
  __syncthreads();
  // the meta granule of every own segment: frames starting in it, the first
  // one's index in the run's list, where its cover is
  {
    // (frames before each own segment: a block-wide exclusive scan of scnt)
    uint64_t* scr = reinterpret_cast<uint64_t*>(L.seg);
    uint64_t carry = 0;
    for (uint64_t i0 = 0; i0 < nown; i0 += G::NT) {
      const uint64_t i = i0 + tid;
      const uint32_t v = i < nown ? I.X.scnt[i] : 0u;
      const uint64_t c = v & 0x7FFFFFFFu;
      uint64_t xs = c;
#pragma unroll
      for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(xs, o, 64);
        if (lane >= o) xs += y;
      }
      if (lane == 63) scr[tid >> 6] = xs;
      __syncthreads();
      uint64_t wb = 0, tot = 0;
      for (uint32_t w = 0; w < G::NT / 64; w++) {
        const uint64_t t = scr[w];
        if (w < (tid >> 6)) wb += t;
        tot += t;
      }
      if (i < nown) {
        const uint64_t before = carry + wb + xs - c;  // own frames starting before this segment
        const uint64_t ss = (s_own0 + i) * TG::SEG;
        uint32_t src = TC_B;
        if (v & 0x80000000u) src = TC_NONE;                           // a frame starts at its first byte
        else if (before || (r == 0 && !na && ss < S0.X)) src = TC_A;  // an own frame (or the carried one) covers it
        st16(P.tdesc + (s_own0 + i) * TD_W,
             uint4{(uint32_t)c, (uint32_t)before, src, 0u});
      }
      carry += tot;
      __syncthreads();
    }
  }
  // end of the workgroup: the last one validates the hand-overs
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t* dn = reinterpret_cast<uint32_t*>(P.tctl + TW_DONE);
    const uint32_t last = atomicAdd(dn, 1u) + 1 == R ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(dn, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    L.done = last;
  }
  __syncthreads();
  if (!L.done) return;
  // --- the finisher (R <= G::NT: one run per thread)
  uint64_t hr = NONE, xr = NONE, nr = 0, ovr = 0, fsr = 0;
  if (tid < R) {
    const uint64_t* rec = P.trec + (uint64_t)tid * TR_WORDS;
    hr = st_load(rec + TR_H); xr = st_load(rec + TR_X); nr = st_load(rec + TR_N);
    ovr = st_load(rec + TR_OVF); fsr = st_load(rec + TR_FS);
  }
  // prev(r): the nearest earlier run with an entry (run 0 always has one:
  // the batch's first frame) — a block-wide inclusive max-scan of the
  // indices of runs with an entry, shifted by one
  int32_t* sc = reinterpret_cast<int32_t*>(L.seg);
  uint64_t* ex = reinterpret_cast<uint64_t*>(L.seg + 4 * G::NT);  // exits by run
  const int32_t me = (tid < R && (hr != NONE || tid == 0)) ? (int32_t)tid : -1;
  sc[tid] = me;
  if (tid < R) ex[tid] = xr;  // (an overflowed run's exit: its first unrecorded frame)
  __syncthreads();
  for (uint32_t o = 1; o < G::NT; o <<= 1) {
    const int32_t y = tid >= o ? sc[tid - o] : -1;
    __syncthreads();
    if (y > sc[tid]) sc[tid] = y;
    __syncthreads();
  }
  // run r's expected entry: the exit of prev(r) = sc[r - 1]. A run whose
  // entry is another position of its range found a false chain (payload
  // bytes that parse as plausible headers); such a chain usually joins the
  // true one within a frame or two (a fake header whose length lands on a
  // true frame start), after which both are the same list: the expected
  // entry among the run's records (a binary search) marks the true frames
  // (the records before it are skipped). Otherwise the run fails (as one
  // without an entry while the chain lands in its range): the batch is
  // covered up to that run's expected entry. After a run whose records
  // overflowed, the next run is not covered.
  uint32_t fail = 0xFFFFFFFFu;
  uint64_t skip = 0, ent = hr;
  if (tid < R && !na) {
    if (tid >= 1) {
      const uint64_t rrb = (uint64_t)tid * P.rbytes, rre = rrb + P.rbytes < P.hi ? rrb + P.rbytes : P.hi;
      const uint64_t expc = ex[sc[tid - 1]];
      if (hr != NONE ? hr != expc : expc < rre) {
        bool joined = false;
        if (hr != NONE && expc < rre && expc > hr && nr) {
          const xyws_frame* list = P.tlist + (uint64_t)tid * P.trcap;
          const int64_t want = (int64_t)(expc - P.lo);
          uint64_t a = 0, b = nr;  // the first record starting at or after expc
          while (a < b) {
            const uint64_t m = (a + b) >> 1;
            if (list[m].frame_off < want) a = m + 1;
            else b = m;
          }
          if (a < nr && list[a].frame_off == want) {
            joined = true;
            skip = a;
            ent = expc;
          }
        }
        if (!joined) fail = tid;
      }
    }
    if (ovr && (hr != NONE || tid == 0)) fail = fail < tid + 1 ? fail : tid + 1;
  }
  if (tid == 0) L.best = 0xFFFFFFFFu;
  __syncthreads();
  if (fail != 0xFFFFFFFFu) atomicMin(&L.best, fail);
  __syncthreads();
  const uint32_t rstar = na ? 0u : (L.best == 0xFFFFFFFFu ? R : (L.best < R ? L.best : R));
  const bool ovfstop = !na && L.best == R;  // (the last run overflowed)
  // ordinal bases (frames of the covered runs before each run) and the total
  const uint64_t c0 = L.aux2;
  {
    uint64_t v = tid < rstar ? nr - skip : 0, xs = v;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(xs, o, 64);
      if (lane >= o) xs += y;
    }
    uint64_t* scr = reinterpret_cast<uint64_t*>(L.seg + 12 * G::NT);
    if (lane == 63) scr[tid >> 6] = xs;
    __syncthreads();
    uint64_t wb = 0, tot = 0;
    for (uint32_t w = 0; w < G::NT / 64; w++) {
      if (w < (tid >> 6)) wb += scr[w];
      tot += scr[w];
    }
    if (tid < R) {
      st_store(P.tctl + TW_BASE + tid, c0 + wb + xs - v);
      st_store(P.tctl + TW_SKIP + tid, skip);
      st_store(P.tctl + TW_ENT + tid, ent);
    }
    if (tid == 0) L.aux1 = c0 + tot;
  }
  // The chain from run 0 is exact up to p, the exit of the last covered run
  // with an entry: past the batch (or a header cut by its end) when every
  // run is covered.
  const int32_t pv = na ? 0 : sc[rstar - 1];
  const uint64_t p = na ? 0 : ex[pv];
  const bool full = !na && !ovfstop && (rstar == R || p >= P.hi);
  if (tid == 0) {
    const xyws_carry* cz = P.cin_user ? P.cin_user : &k_zero_carry;
    uint64_t* rd = P.lat + LW_REDIR;
    const uint64_t total = L.aux1;
    const uint64_t E = L.E;
    st_store(P.tctl + TW_EPOCH, E);
    if (na) {
      st_store(P.tctl + TW_PCOV, 0);
      st_store(rd, RD_FULL);
    } else {
      lat_carried_frame(P, cz);
      if (!full) {
        // the run decoder takes the batch from p as a fresh stream, counting
        // on from the frames before it
        st_store(P.tctl + TW_PCOV, p);
        uint64_t* rc = P.lat + LW_RCARRY;
#pragma unroll
        for (int i = 0; i < 8; i++) st_store(rc + i, 0);
        st_store(rc + 2, cz->frames_total + total);
        st_store(rd + 1, p);
        st_store(rd + 2, total);
        st_store(rd, RD_FROM);
      } else {
        st_store(P.tctl + TW_PCOV, P.hi);
        const cstate S = get_state(P.trec + (uint64_t)pv * TR_WORDS + TR_S);
        xyws_carry cinc;
#pragma unroll
        for (int i = 0; i < 8; i++) reinterpret_cast<uint64_t*>(&cinc)[i] = reinterpret_cast<const uint64_t*>(cz)[i];
        write_outputs(P, &cinc, total, S);
        st_store(rd, RD_DONE);
      }
      // The frame covering [its start, p): the last frame of run pv (or the
      // carried one). The stream kernel takes it as the covering frame of
      // every segment of the runs not covered (from rstar on, up to p):
      // their cover slot B may hold a false chain's frame (a run past the
      // first mismatch writes there too), the true one is this.
      const uint64_t npv = st_load(P.trec + (uint64_t)pv * TR_WORDS + TR_N);
      uint64_t tps = 0, tpe = 0, tkw = 0;
      if (npv) {
        const xyws_frame f = P.tlist[(uint64_t)pv * P.trcap + npv - 1];
        tps = (uint64_t)f.payload_off + P.lo;
        const uint64_t e = sat_add(tps, f.payload_len);
        tpe = e < P.hi ? e : P.hi;
        const uint32_t key = (uint32_t)f.key[0] | ((uint32_t)f.key[1] << 8) | ((uint32_t)f.key[2] << 16) |
                             ((uint32_t)f.key[3] << 24);
        tkw = aligned_key(key, tps, 0);
      } else if (!(S0.st & S_NOCOV)) {
        tps = S0.cov_ps;
        tpe = S0.X < P.hi ? S0.X : P.hi;
        tkw = S0.cov_kw;
      }
      st_store(P.tctl + TW_TAIL, tps);
      st_store(P.tctl + TW_TAIL + 1, tpe);
      st_store(P.tctl + TW_TAIL + 2, tkw);
    }
    st_store(P.tctl + TW_RSTAR, rstar);
  }
  // decoder-choice words: the last frame of every covered run (as the run
  // decoder's runs report theirs); published only when everything is covered
  // (else the run decoder after the stream kernel publishes)
  if (full && tid < rstar && fsr) fs_note(P, fsr, fsr);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0 && full) pol_publish(P, L.E, DEC_TABLE);
}

// ---------------------------------------------------------------- the stream
template <class TG>
struct __attribute__((aligned(16))) tab_lds {
  uint8_t seg[TG::SEG + 48];
  uint4 tab[TG::NMAX + 2];  // the segment's frames: {payload start, payload end, key word, 0}, sorted
  uint4 dsc[TD_W];          // the segment's descriptor (loaded one segment ahead by the claim wave)
  uint64_t rsk[2];          // its run's skipped records and first true frame start (TW_SKIP, TW_ENT)
  uint64_t pcov, tps, tpe;
  uint32_t tkw, rstar, nsegc, cur, nxt, done_last;
};

// XOR mask of the 16-byte chunk at segment offset a: the frames it overlaps
// (sorted by payload start; the last one starting at or before a, found by
// a binary search, and the ones after it starting inside the chunk).
XYWS_DEV u32x4 tab_mask(const uint4* tab, uint32_t nent, uint32_t a) {
  uint32_t lo = 0, hi = nent;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (tab[mid].x <= a) lo = mid;
    else hi = mid;
  }
  const uint4 g = tab[lo];
  if (g.x <= a && a + 16u <= g.y) return u32x4{g.z, g.z, g.z, g.z};
  u32x4 m = span_key16(a, g.x, g.y, g.z);
  for (uint32_t j = lo + 1; j < nent; j++) {
    const uint4 n = tab[j];
    if (n.x >= a + 16u) break;
    m |= span_key16(a, n.x, n.y, n.z);
  }
  return m;
}

// Stream kernel (see the file comment): segments [0, nsegc) (those holding a
// byte below the coverage end p), claimed as in the lattice decoder (a static
// first round, then one counter, one claim ahead); every wave moves rows.
template <class TG>
__global__ void __launch_bounds__(TG::NT) k_stream_table(run_params P) {
  constexpr uint32_t NW = TG::NT / 64, NROW = TG::SEG / 1024, K = NROW / NW;
  extern __shared__ __attribute__((aligned(16))) uint8_t xs_lds[];
  tab_lds<TG>& L = *reinterpret_cast<tab_lds<TG>*>(xs_lds);
  uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(P.tctl + TW_CLAIM);
  if (tid == 0) {
    const uint64_t pc = st_load(P.tctl + TW_PCOV);
    L.pcov = pc;
    L.rstar = (uint32_t)st_load(P.tctl + TW_RSTAR);
    L.tps = st_load(P.tctl + TW_TAIL);
    L.tpe = st_load(P.tctl + TW_TAIL + 1);
    L.tkw = (uint32_t)st_load(P.tctl + TW_TAIL + 2);
    const uint64_t n = (pc + TG::SEG - 1) / TG::SEG;
    L.nsegc = (uint32_t)n;
    L.cur = blockIdx.x < n ? blockIdx.x : NONE32;
  }
  __syncthreads();
  const uint64_t pcov = L.pcov;
  const uint32_t rstar = L.rstar, nsegc = L.nsegc;
  uint32_t cur = L.cur;
  uint32_t ahead = blockIdx.x - gridDim.x;  // claim lane: (+ 2 * grid at its use: the static b + grid)
  u32x4 e[K];
  u32x4 dv = {0u, 0u, 0u, 0u};  // claim wave: a granule of the descriptor, or (lanes 16, 17) the run's words
  auto issue = [&](uint32_t s, bool claim) {
    if (wave == 0) {
      if (lane == 0) {
        if (claim)
          asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(ahead) : "v"(cnt), "v"(1u) : "memory");
        else
          ahead = LAT_NOCLAIM;
      }
      if (lane < TD_W) {
        dv = *reinterpret_cast<const u32x4*>(P.tdesc + (uint64_t)s * TD_W + lane);
      } else if (lane < TD_W + 2) {
        const uint64_t v = P.tctl[(lane == TD_W ? TW_SKIP : TW_ENT) + s / P.tspr];
        dv = u32x4{(uint32_t)v, (uint32_t)(v >> 32), 0u, 0u};
      }
    }
    const __amdgpu_buffer_rsrc_t rs = lat_rsrc(P, (uint64_t)s * TG::SEG, TG::SEG);
#pragma unroll
    for (uint32_t k = 0; k < K; k++)
      e[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16u, (wave + NW * k) * 1024u, AUX_NT);
  };
  if (cur != NONE32) {
    const uint32_t a0 = ahead;
    issue(cur, false);
    ahead = a0;
    const __amdgpu_buffer_rsrc_t rs = lat_rsrc(P, (uint64_t)cur * TG::SEG, TG::SEG);
#pragma unroll
    for (uint32_t k = 0; k < K; k++)
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, rs, OOB, k * 1024u, AUX_ST_STREAM);
  }
  while (cur != NONE32) {
    asm volatile("" : "+v"(tid));
    const uint64_t ss = (uint64_t)cur * TG::SEG;
    __syncthreads();  // (A) the previous segment's LDS reads are done
#pragma unroll
    for (uint32_t k = 0; k < K; k++) *reinterpret_cast<u32x4*>(&L.seg[(wave + NW * k) * 1024u + lane * 16u]) = e[k];
    if (wave == 0) {
      asm volatile("" : "+v"(ahead), "+v"(dv) : "v"(e[K - 1].x));
      if (lane < TD_W) *reinterpret_cast<u32x4*>(&L.dsc[lane]) = dv;
      else if (lane < TD_W + 2) L.rsk[lane - TD_W] = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
      if (lane == 0) {
        const uint32_t a = ahead + 2u * gridDim.x;
        L.nxt = a < nsegc ? a : NONE32;
      }
    }
    __syncthreads();  // (B)
    const uint32_t nxt = L.nxt;
    if (nxt != NONE32) issue(nxt, true);
    // the segment's table: the covering frame, then the frames starting in it
    const uint4 meta = L.dsc[0];
    const uint64_t r = cur / P.tspr;
    const bool own = r < rstar;
    const uint32_t n = own ? meta.x : 0u, lo = meta.y;
    const uint64_t skip = L.rsk[0], ent = L.rsk[1];
    uint32_t first = lo, cnt = n, src = meta.z;
    if (skip && skip >= lo) {
      // records of a false chain (before the run's first true frame): no true
      // frame of the run starts before this segment
      const uint32_t drop = skip - lo < n ? (uint32_t)(skip - lo) : n;
      first = lo + drop;
      cnt = n - drop;
      src = ent == ss ? TC_NONE : TC_B;
    }
    if (tid == 0)
      L.tab[0] = !own ? tab_entry(L.tps, L.tpe, L.tkw, ss)  // (a run not covered: the last exact frame)
                 : src == TC_A ? L.dsc[2] : src == TC_B ? L.dsc[1] : uint4{0u, 0u, 0u, 0u};
    const uint32_t in0 = first - lo;  // (the first inline slot used)
    for (uint32_t i = tid; i < cnt; i += TG::NT) {
      if (in0 + i < TD_K) {
        L.tab[1 + i] = L.dsc[3 + in0 + i];
      } else {
        // (rare: more frames start in the segment than its descriptor holds)
        const xyws_frame f = P.tlist[r * P.trcap + first + i];
        const uint64_t ps = (uint64_t)f.payload_off + P.lo, end = sat_add(ps, f.payload_len);
        const uint32_t key = (uint32_t)f.key[0] | ((uint32_t)f.key[1] << 8) | ((uint32_t)f.key[2] << 16) |
                             ((uint32_t)f.key[3] << 24);
        L.tab[1 + i] = tab_entry(ps, end < P.hi ? end : P.hi, aligned_key(key, ps, 0), ss);
      }
    }
    __syncthreads();  // (C) the table is complete
    // stores: each chunk XORed with the keys of the frames it overlaps, up to
    // the coverage end (the run decoder's bytes after it are left as they are)
    const uint32_t nent = 1u + cnt;
    const uint32_t lo_r = lat_rel(P.lo, ss), hi_r = P.hi - ss < TG::SEG ? (uint32_t)(P.hi - ss) : TG::SEG;
    const uint32_t stop = pcov - ss < TG::SEG ? (uint32_t)(pcov - ss) : TG::SEG;
    const __amdgpu_buffer_rsrc_t rs = lat_rsrc(P, ss, TG::SEG);
    uint32_t edge = 0;
    u32x4 dprev = {0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t k = 0; k < K; k++) {
      const uint32_t a = (wave + NW * k) * 1024u + lane * 16u;
      u32x4 d = *reinterpret_cast<const u32x4*>(&L.seg[a]);
      d = d ^ tab_mask(L.tab, nent, a);
      const bool whole = a >= lo_r && a + 16u <= hi_r && a + 16u <= stop;
      if (!whole && a < stop && a < hi_r && a + 16u > lo_r) {
        edge |= 1u << k;
        *reinterpret_cast<u32x4*>(&L.seg[a]) = d;  // (stored bytewise below)
      }
      __builtin_amdgcn_raw_buffer_store_b128(d, rs, whole ? lane * 16u : OOB, (wave + NW * k) * 1024u, AUX_ST_STREAM);
      asm volatile("" ::"v"(dprev.x), "v"(dprev.y), "v"(dprev.z), "v"(dprev.w));
      dprev = d;
    }
    asm volatile("s_nop 1" ::"v"(dprev.x), "v"(dprev.y), "v"(dprev.z), "v"(dprev.w));
#pragma nounroll
    while (edge) {
      const uint32_t k = __builtin_ctz(edge);
      edge &= edge - 1;
      const uint32_t a = (wave + NW * k) * 1024u + lane * 16u;
#pragma nounroll
      for (uint32_t y = a; y < a + 16u; y++)
        if (y >= lo_r && y < hi_r && y < stop) P.base[ss + y] = L.seg[y];
    }
    cur = nxt;
  }
  // end: the last workgroup resets the claim counter for the next call
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    uint32_t* dn = reinterpret_cast<uint32_t*>(P.tctl + TW_DONE) + 1;
    if (atomicAdd(dn, 1u) + 1 == gridDim.x) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dn, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Descriptors (the caller asked for them): workgroup r copies run r's
// records to their ordinals, for the covered runs.
__global__ void __launch_bounds__(256) k_table_emit(run_params P) {
  const uint32_t r = blockIdx.x;
  if (r >= (uint32_t)st_load(P.tctl + TW_RSTAR)) return;
  const uint64_t n = st_load(P.trec + (uint64_t)r * TR_WORDS + TR_N);
  const uint64_t base = st_load(P.tctl + TW_BASE + r), skip = st_load(P.tctl + TW_SKIP + r);
  const xyws_frame* list = P.tlist + (uint64_t)r * P.trcap;
  for (uint64_t i = skip + threadIdx.x; i < n; i += 256) {
    const uint64_t ord = base + i - skip;
    if (ord >= P.cap) break;
    P.frames[ord] = list[i];
  }
}
