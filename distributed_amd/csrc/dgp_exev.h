// The vector-form executor (exe_v): what exe_local does for an F_FAST stimulus on the LDS
// worker layout, written so that one stimulus is a short VALU program.
//
// Why (profiles/r05g, one executor, per-phase s_memtime stamps): a local stimulus took ~20k
// cycles on one wave although it issues well under 2k instructions; the time went to chains
// of VALU -> SGPR -> SALU -> VALU crossings (readlane of a descriptor entry, a scalar compare,
// v_cmp into an SGPR mask, a branch on it, again per dependency): the first commit's
// needs_what update alone took 1.8k cycles, its dict update 1.4k. Here every per-worker or
// per-dependency step is one lane's straight-line VALU work with selects instead of branches
// (a lane = a touched worker, or a descriptor entry = a dependency), and the uniform values
// cross to scalars once each:
//  * needs_what (:800-823): each dependency's lane reads the worker's whole LDS line (three
//    broadcast ds_read_b128), finds its entry by compare-and-select, and writes its own entry
//    back (a task's dependencies are distinct, so their entries are distinct words);
//  * the prefix dict (:733-784): insertion-ordered slots updated by selects on every lane, the
//    result kept on the one lane it is for;
//  * decide_worker's argmin (:8550-8593, worker_objective :3131-3146): PRE's per-candidate
//    comm / bandwidth (frow rows) added to each lane's stack time, one row-wide DPP minimum of
//    the order-preserving start key; ties (equal start) fall to the exact serial key.
// Nothing is written to LDS before the wait for the frontier candidates is over and their
// needs tables are known to fit: a stimulus this path cannot take returns false unchanged and
// exe_local runs it instead (overflowing needs_what lines, replica events it does not model).
// Reference semantics, operation order and fp64 arithmetic are exe_local's (bit-exact).

namespace ev {

// the 8 insertion-ordered slots of a worker's prefix dict as an array (constant indices only)
struct VDict {
  uint32_t s[PD];
  uint32_t n;  // entries
};
__device__ __forceinline__ VDict vd_of(const WDict& d) {
  VDict v;
  v.s[0] = d.c.x; v.s[1] = d.c.y; v.s[2] = d.c.z; v.s[3] = d.c.w;
  v.s[4] = d.c1.x; v.s[5] = d.c1.y; v.s[6] = d.c1.z; v.s[7] = d.c1.w;
  v.n = d.ord >> 24;
  return v;
}
__device__ __forceinline__ WDict wd_of(const VDict& v) {
  WDict d;
  d.c = make_uint4(v.s[0], v.s[1], v.s[2], v.s[3]);
  d.c1 = make_uint4(v.s[4], v.s[5], v.s[6], v.s[7]);
  d.ord = v.n << 24;
  return d;
}

// add_to_processing (+1) of prefix p on the lanes with `sel` (:733-745); false on a lane whose
// count would overflow or whose dict is full (the caller raises SERR_PREFIX)
__device__ __forceinline__ bool vd_inc(VDict& v, bool sel, int p) {
  const uint32_t pk = (uint32_t)p;
  bool found = false, sat = false;
  uint32_t t[PD];
#pragma unroll
  for (int i = 0; i < PD; i++) {
    const bool m = (uint32_t)i < v.n && (v.s[i] >> 24) == pk;
    found = found || m;
    sat = sat || (m && (v.s[i] & 0xffffffu) == 0xffffffu);
    t[i] = m ? v.s[i] + 1u : v.s[i];
  }
#pragma unroll
  for (int i = 0; i < PD; i++) t[i] = (!found && (uint32_t)i == v.n) ? ((pk << 24) | 1u) : t[i];
  const bool ok = found ? !sat : (v.n < (uint32_t)PD && p >= 0 && p <= 255);
  const bool ap = sel && ok;
#pragma unroll
  for (int i = 0; i < PD; i++) v.s[i] = ap ? t[i] : v.s[i];
  v.n = (ap && !found) ? v.n + 1u : v.n;
  return !sel || ok;
}

// remove_from_processing (-1) of prefix p on the lanes with `sel` (:760-771): the count drops,
// at zero the key leaves and later keys move up
__device__ __forceinline__ void vd_dec(VDict& v, bool sel, int p) {
  const uint32_t pk = (uint32_t)p;
  int k = PD;  // the slot of p (PD: absent)
  uint32_t ck = 0;
#pragma unroll
  for (int i = PD - 1; i >= 0; i--) {
    const bool m = (uint32_t)i < v.n && (v.s[i] >> 24) == pk;
    k = m ? i : k;
    ck = m ? (v.s[i] & 0xffffffu) : ck;
  }
  const bool hit = sel && k < PD;
  const bool gone = hit && ck <= 1u;
  uint32_t t[PD];
#pragma unroll
  for (int i = 0; i < PD; i++) {
    const uint32_t nx = i + 1 < PD ? v.s[i + 1] : 0u;
    t[i] = gone ? (i >= k ? nx : v.s[i]) : ((hit && i == k) ? v.s[i] - 1u : v.s[i]);
  }
#pragma unroll
  for (int i = 0; i < PD; i++) v.s[i] = t[i];
  v.n = gone ? v.n - 1u : v.n;
}

// _calc_occupancy (:1884-1903) on every lane: the prefix terms in dict order, then the network
// term (netocc / bandwidth, carried per lane); the same fp64 operations as occ_dict_r. `nm`
// (uniform) bounds every lane's entry count.
__device__ __forceinline__ double vd_occ(const VDict& v, int nm, double net_bw, DTab dt, const Dev& D) {
  double dv[PD];
#pragma unroll
  for (int i = 0; i < PD; i++)
    if (i < nm) dv[i] = dt[(v.s[i] >> 24) & (PX - 1)];  // every load issued before the sum
  double res = 0.0;
#pragma unroll
  for (int i = 0; i < PD; i++) {
    if (i >= nm) break;
    const double term = (dv[i] < 0 ? D.unknown_duration : dv[i]) * (double)(v.s[i] & 0xffffffu);
    res = (uint32_t)i < v.n ? res + term : res;
  }
  return res + net_bw;
}

// maximum over lanes 0..15 (DPP within row 0), uniform
__device__ __forceinline__ int row0_max(int v) {
  v = max(v, __builtin_amdgcn_update_dpp(v, v, 0xb1, 0xf, 0xf, false));   // quad_perm(1,0,3,2)
  v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x4e, 0xf, 0xf, false));   // quad_perm(2,3,0,1)
  v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x140, 0xf, 0xf, false));  // row_mirror
  return rl(v, 0);
}

// one worker's needs_what line (words 0..NLW-2 entries d << 8 | count, NLW-1 control), read
// whole into every lane (three broadcast 16-byte LDS reads)
struct Line {
  uint32_t e[NLW];
};
template <bool LW>
__device__ __forceinline__ Line line_all(const WPtr<LW>& P, int c) {
  static_assert(NLW == 12, "three 16-byte words");
  using U4 = typename WPtr<LW>::template P<const Q4>;
  const U4 q = ascast<U4>(P.needs + (size_t)c * NLW);
  const uint4 a = ld4(q), b = ld4(q + 1), d = ld4(q + 2);
  Line l;
  l.e[0] = a.x; l.e[1] = a.y; l.e[2] = a.z; l.e[3] = a.w;
  l.e[4] = b.x; l.e[5] = b.y; l.e[6] = b.z; l.e[7] = b.w;
  l.e[8] = d.x; l.e[9] = d.y; l.e[10] = d.z; l.e[11] = d.w;
  return l;
}
// the entry of dependency d in the line (NLW - 1: none)
__device__ __forceinline__ int line_find(const Line& l, uint32_t d, uint32_t& val) {
  int m = NLW - 1;
  val = 0;
#pragma unroll
  for (int i = NLW - 2; i >= 0; i--) {
    const bool h = l.e[i] != 0u && (l.e[i] >> 8) == d;
    m = h ? i : m;
    val = h ? l.e[i] : val;
  }
  return m;
}
// a line the vector form updates in place: every entry in the LDS words (count == words in
// use: no overflow entries in D.gw_needs_ext), not in scan mode
__device__ __forceinline__ bool line_plain(const Line& l) {
  int used = 0;
#pragma unroll
  for (int i = 0; i < NLW - 1; i++) used += l.e[i] != 0u ? 1 : 0;
  const uint32_t ctl = l.e[NLW - 1];
  return ctl != NL_OVF && (int)(ctl >> 8) == used;
}

// sum over the lanes of mask m of an int64 held per lane (few lanes: serial on scalars)
__device__ __forceinline__ int64_t msum64(unsigned long long m, int64_t v) {
  int64_t s = 0;
  for (; m; m &= m - 1) s += rl_i64(v, __builtin_ctzll(m));
  return s;
}

}  // namespace ev

// exe_v: an F_FAST stimulus (local, at most NFF frontier tasks, none restricted, at most TF
// touched workers, P <= PD) with its state in LDS. false: nothing changed, run exe_local.
template <bool LW>
__device__ __attribute__((always_inline)) bool exe_v(const Dev& D, SLds& L, const WPtr<LW>& P, int s, long long r,
                                                     int qmode, const uint4& E, int& woke) {
  using namespace ev;
  using U4 = typename WPtr<LW>::template P<Q4>;
  SCtl& S = L.c;
  const int lane = lane_id();
  // PRE's frontier-candidate rows (comm / bandwidth, comm per touched worker): in flight while
  // the touched workers' state is read
  const uint4* FRr = D.frow + (size_t)(r & (DR - 1)) * FRS;
  const bool l16 = lane < TF;
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  uint4 FJ[NFF];
#pragma unroll
  for (int j = 0; j < NFF; j++) FJ[j] = l16 ? FRr[j * TF + lane] : z4;
  // ---- the touched workers (entry 0 = w), one lane each, and their state
  const int nt = L.ntouch[s];
  const bool tl = lane < nt;
  const int tv = tl ? (int)L.touch[s][lane] : 0;
  const int cj = tv & T_W;
  const bool candl = (tv & T_CAND) != 0;
  const bool wc = WAITC && tl && lane > 0 && candl;  // candidate-only: read after the wait
  int np = 0, nth = 1;
  uint32_t ctl = 0;
  WDict dw;
  dw.c = z4;
  dw.c1 = z4;
  dw.ord = 0;
  int64_t net = 0, nbj = 0;
  if (tl) {
    nth = P.nthreads[cj];
    ctl = P.needs[(size_t)cj * NLW + NLW - 1];
    np = P.nproc[cj];
    dw = dict_load<LW>(P, cj);
    net = P.netocc[cj];
    nbj = P.nbytes[cj];
  }
  const DTab durv = stim_durations(D, L, E, r);
  const int t = rl((int)E.x, 0), w = rl((int)E.y, 0), p = rl((int)E.z, 0);
  const uint32_t flags = rlu(E.w, 0);
  const int64_t nbt = mk64(rlu(E.x, 1), rlu(E.y, 1));
  const unsigned cnts = rlu(E.z, 1);
  const int kt = cnts & 0xff, nrel = (cnts >> 8) & 0xff, nf = (cnts >> 16) & 0xff;
  const double dobs = mkd(rlu(E.x, 2), rlu(E.y, 2));
  const int tot_new = rl((int)E.w, 2);  // needs_what entries the frontier may add (PRE)
  const int TD = E_HDR, RL0 = E_HDR + kt, FX0 = RL0 + nrel;
  const int capw = P.cap[w];
  // capacity of the needs tables this stimulus may grow (exe_local's check; a candidate-only
  // worker's may still grow by earlier stimuli: with a margin now, exactly after the wait)
  {
    const int slack = wc ? NXW / 2 : 0;
    if (ballot(tl && (ctl == NL_OVF || (int)(ctl >> 8) + tot_new + slack > NLW - 1 + NXW))) return false;
  }
  if (nt < 1 || rl(cj, 0) != w) {
    serr(S, SERR_INV, 700000000 + (int)r);
    return true;
  }
  if (TR3 && lane == 0) {
    TR(r, 8);
    trace_at(D, r, 22, (unsigned long long)(nf | kt << 8 | nrel << 16 | nt << 24));
  }
  const bool isw = lane == 0;
  const bool nth1 = !ballot(tl && nth != 1);  // occ / 1.0 == occ: the division is skipped
  // ---- completion: processing -> memory (:2366): _dec_needs_replica for every dependency
  // of t that w does not hold (:815-823); a dependency's lane finds its entry in w's line
  const bool dl = lane >= TD && lane < TD + kt && (int)E.y != w;
  uint32_t dval = 0, ctlw = 0;
  int dm = NLW - 1;
  bool wplain;
  {
    const Line lw = line_all<LW>(P, w);
    wplain = line_plain(lw);
    ctlw = lw.e[NLW - 1];
    if (dl) dm = line_find(lw, E.x, dval);
  }
  // an entry not in the line (replica events, exe_local's general path): exe_local
  if (wplain && ballot(dl && dm == NLW - 1)) return false;
  const bool dgone = wplain && dl && (dval & 0xffu) == 1u;
  const unsigned long long gm = ballot(dgone);
  const int ngone = __builtin_popcountll(gm);
  int64_t dnet = -msum64(gm, mk64(E.z, E.w));
  const int npw = rl(np, 0) - 1;
  if (TR3 && lane == 0) TR(r, 10);
  // ---- the wait for the candidates (WAITC): every earlier stimulus holding one has released it
  int nm = row0_max(tl ? (int)(dw.ord >> 24) : 0);
  bool released = false;
  if (TR3 && lane == 0) TR(r, 11);
  if (WAITC && ballot(wc)) {
    if (vload(&L.predc[s]) != 0) {
      if (DGP_EXE_PRIO) __builtin_amdgcn_s_setprio(1);
      while (vload(&L.predc[s]) != 0) __builtin_amdgcn_s_sleep(1);
      if (DGP_EXE_PRIO) __builtin_amdgcn_s_setprio(3);
    }
    lds_fence();
    if (wc) {
      ctl = P.needs[(size_t)cj * NLW + NLW - 1];
      np = P.nproc[cj];
      dw = dict_load<LW>(P, cj);
      net = P.netocc[cj];
      nbj = P.nbytes[cj];
    }
    // (exe_local continues such a stimulus as the oldest, exact; nothing is written yet here)
    if (ballot(wc && (ctl == NL_OVF || (int)(ctl >> 8) + tot_new > NLW - 1 + NXW))) return false;
    nm = row0_max(tl ? (int)(dw.ord >> 24) : 0);
  }
  // ================= committed: from here on this path finishes the stimulus
  if (TR3 && lane == 0) TR(r, 12);
  OutR o;
  o.init();
  // w's line: the completion's entries, then the control word (count of entries)
  if (wplain) {
    if (dl) P.needs[(size_t)w * NLW + dm] = dgone ? 0u : dval - 1u;
    if (npw == 0) {  // a worker with nothing processing needs nothing (needs_reset)
      if (lane < NLW) P.needs[(size_t)w * NLW + lane] = 0u;
    } else if (ngone && lane == 0) {
      P.needs[(size_t)w * NLW + NLW - 1] = ctlw - ((uint32_t)ngone << 8);
    }
  } else {  // overflow entries: exe_local's one-at-a-time form
    uint32_t nl = line_load<LW>(P, w);
    for (int i = 0; i < kt; i++) {
      const int L_ = TD + i;
      if (rl((int)E.y, L_) == w) continue;
      dnet -= needs_dec(D, S, w, nl, rl((int)E.x, L_), mk64(rlu(E.z, L_), rlu(E.w, L_)), t);
    }
    if (npw == 0) needs_reset(D, w, nl);
    line_store<LW>(P, w, nl);
  }
  VDict dj = vd_of(dw);
  vd_dec(dj, isw, p);
  if (isw) {
    np = npw;
    net += dnet;
  }
  double nbw = (double)net / (double)D.bandwidth;  // net_bw_of
  double occj = vd_occ(dj, nm, nbw, durv, D);
  double stkj = nth1 ? occj : occj / (double)nth;
  o.rec(K_COMPLETE, w, p, dnet, rl_f64(occj, 0), npw, t, dobs);
  // add_replica (:3148), then the releases popped before the frontier (LIFO, :3309-3314)
  if (isw) nbj += (flags & F_SELFREL) ? 0 : nbt;
  for (int i = 0; i < nrel; i++) {
    const int h = rl((int)E.x, RL0 + i);
    const int64_t nb = mk64(rlu(E.z, RL0 + i), rlu(E.w, RL0 + i));
    nbj = (tl && cj == h) ? nbj - nb : nbj;
  }
  {  // a release-only holder (ws.nbytes of a released dependency) is final now
    const bool ro = tl && !isw && !candl;
    if (ballot(ro)) {
      if (ro) P.nbytes[cj] = nbj;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the state above is in LDS
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      if (ro) release_worker<LW>(L, P, s, cj);
      released = ro;
    }
  }
  // ------------------------------ frontier in ascending priority: decide_worker (:8550)
  if (TR3 && lane == 0) TR(r, 13);
  int off = FX0;
#pragma unroll 1
  for (int j = 0; j < nf; j++) {
    const uint4 FR = j == 0 ? FJ[0] : j == 1 ? FJ[1] : j == 2 ? FJ[2] : FJ[3];
    const int x = rl((int)E.x, off), px = rl((int)E.y, off);
    const int kx = rl((int)E.z, off) & 0xff;
    const unsigned cmask = rlu(E.w, off);  // the candidates' touch indices (PRE)
    // worker_objective (:3131-3146): start = occupancy / nthreads + comm_bytes / bandwidth,
    // then (start, ws.nbytes, canonical index) minimal over the candidates
    const bool cand = tl && ((cmask >> lane) & 1u);
    const double start = stkj + mkd(FR.x, FR.y);
    const uint64_t sk = cand ? start_key(start) : ~0ull;
    const uint64_t mk = rl64(row_min_u64(sk), 0);
    const unsigned long long eq = ballot(cand && sk == mk);
    if (!eq) {
      serr(S, SERR_CAND, x);
      return true;
    }
    int jb = __builtin_ctzll(eq);
    if (eq & (eq - 1)) {  // equal start times: ws.nbytes, then the worker index (key_less)
      int64_t bn = rl_i64(nbj, jb);
      int bw = rl(cj, jb);
      for (unsigned long long m = eq & (eq - 1); m; m &= m - 1) {
        const int q = __builtin_ctzll(m);
        const int64_t nq = rl_i64(nbj, q);
        const int wq = rl(cj, q);
        if (nq < bn || (nq == bn && wq < bw)) {
          jb = q;
          bn = nq;
          bw = wq;
        }
      }
    }
    const int cb = rl(cj, jb);
    const double bstart = rl_f64(start, jb);
    const int64_t bnb = rl_i64(nbj, jb);
    const int64_t bcomm = mk64(rlu(FR.z, jb), rlu(FR.w, jb));
    if (j == nf - 1 && nt > 2) {
      // the last frontier decision is made: every touched worker but w and the chosen one is
      // final now; written back and released before the commit
      const bool early = tl && !isw && lane != jb && !released;
      if (ballot(early)) {
        if (early) {
          const WDict d2 = wd_of(dj);
          P.nproc[cj] = np;
          st4(ascast<U4>(P.pcnt + (size_t)cj * PD), d2.c);
          st4(ascast<U4>(P.pcnt + (size_t)cj * PD + 4), d2.c1);
          P.plen[cj] = d2.ord;
          P.netocc[cj] = net;
          P.nbytes[cj] = nbj;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the state above is in LDS
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (early) release_worker<LW>(L, P, s, cj);
        released = released || early;
      }
    }
    // _add_to_processing (:3199): record, WorkerState.add_to_processing (_inc_needs_replica
    // :800-813 for the dependencies cb does not hold), check_idle_saturated
    if (TR3 && lane == 0 && j == 0) TR(r, 14);
    o.place(x, cb, bcomm, bstart, bnb, ROUTE_NONROOTISH);
    const bool xl = lane > off && lane <= off + kx && (int)E.y != cb;  // x's dependency lanes
    int64_t dn = 0;
    const Line lc = line_all<LW>(P, cb);
    // the vector form: every dependency's entry found or given the lowest free word (in
    // dependency order); a line with overflow entries, or without the free words, takes
    // exe_local's one-at-a-time form (nothing written before the choice)
    if (TR3 && lane == 0 && j == 0) { __builtin_amdgcn_s_waitcnt(0xc07f); TR(r, 24); }
    uint32_t val = 0;
    const int m = xl ? line_find(lc, E.x, val) : NLW - 1;
    const bool hit = xl && m < NLW - 1;
    const bool ins = xl && !hit;
    const unsigned long long im = ballot(ins);
    const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(im >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)im, 0u));
    int slot = NLW - 1, nfree = 0;
#pragma unroll
    for (int i = 0; i < NLW - 1; i++) {
      const bool fr = lc.e[i] == 0u;
      slot = (fr && nfree == rank && slot == NLW - 1) ? i : slot;
      nfree += fr ? 1 : 0;
    }
    const bool vec = line_plain(lc) && !ballot(ins && slot == NLW - 1) && !ballot(hit && (val & 0xffu) == 0xffu);
    if (vec) {
      const int nins = __builtin_popcountll(im);
      if (hit) P.needs[(size_t)cb * NLW + m] = val + 1u;
      if (ins) P.needs[(size_t)cb * NLW + slot] = (E.x << 8) | 1u;
      if (nins && lane == 0) P.needs[(size_t)cb * NLW + NLW - 1] = lc.e[NLW - 1] + ((uint32_t)nins << 8);
      dn = msum64(im, mk64(E.z, E.w));
    } else {  // exe_local's one-at-a-time form (overflow entries in D.gw_needs_ext)
      uint32_t nlc = line_load<LW>(P, cb);
      for (int i = 0; i < kx; i++) {
        const int L2 = off + 1 + i;
        if (rl((int)E.y, L2) == cb) continue;
        dn += needs_inc(D, S, cb, nlc, rl((int)E.x, L2), mk64(rlu(E.z, L2), rlu(E.w, L2)), x);
      }
      line_store<LW>(P, cb, nlc);
    }
    if (TR3 && lane == 0 && j == 0) TR(r, 25);
    const bool isb = lane == jb;
    if (ballot(!vd_inc(dj, isb, px))) serr(S, SERR_PREFIX, x);
    if (TR3 && lane == 0 && j == 0) TR(r, 26);
    nm = min(nm + 1, PD);
    if (isb) {
      np += 1;
      net += dn;
      if (dn != 0) nbw = (double)net / (double)D.bandwidth;
    }
    occj = vd_occ(dj, nm, nbw, durv, D);
    stkj = nth1 ? occj : occj / (double)nth;
    if (TR3 && lane == 0 && j == 0) TR(r, 27);
    o.rec(K_PLACE, cb, px, dn, rl_f64(occj, jb), rl(np, jb), x, 0.0);
    off += 1 + kx;
    if (TR3 && lane == 0 && j == 0) TR(r, 15);
  }
  if (TR3 && lane == 0) TR(r, 16);
  // ---- every touched worker but w is final: written back and released
  if (tl && !isw && !released) {
    const WDict d2 = wd_of(dj);
    P.nproc[cj] = np;
    st4(ascast<U4>(P.pcnt + (size_t)cj * PD), d2.c);
    st4(ascast<U4>(P.pcnt + (size_t)cj * PD + 4), d2.c1);
    P.plen[cj] = d2.ord;
    P.netocc[cj] = net;
    P.nbytes[cj] = nbj;
  }
  if (nt > 1) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (tl && !isw && !released) release_worker<LW>(L, P, s, cj);
  }
  // -------------- stimulus_queue_slots_maybe_opened (:4983): only w can have open slots
  if (TR3 && lane == 0) TR(r, 17);
  int pops = 0;
  if (qmode != 0 && !D.sat_inf) {
    const int slots = capw - rl(np, 0);
    if (slots > capw || o.npl + slots > PLC - 1) {
      serr(S, SERR_INV, 600000000 + (int)r);
      return true;
    }
    if (slots > 0) pops = slots;
    const int qp = S.q_prefix;
    const int64_t nbw0 = rl_i64(nbj, 0);
    for (int i = 0; i < pops; i++) {
      const double st = stkj + 0.0 / (double)D.bandwidth;
      o.place(-1, w, 0, rl_f64(st, 0), nbw0, ROUTE_ROOTISH_Q);
      if (ballot(!vd_inc(dj, isw, qp))) serr(S, SERR_PREFIX, -1);
      nm = min(nm + 1, PD);
      if (isw) np += 1;
      occj = vd_occ(dj, nm, nbw, durv, D);
      stkj = nth1 ? occj : occj / (double)nth;
      o.rec(K_PLACE, w, qp, 0, rl_f64(occj, 0), rl(np, 0), -1, 0.0);
    }
  }
  // ---- w written back last, then released
  if (isw) {
    const WDict d2 = wd_of(dj);
    P.nproc[cj] = np;
    st4(ascast<U4>(P.pcnt + (size_t)cj * PD), d2.c);
    st4(ascast<U4>(P.pcnt + (size_t)cj * PD + 4), d2.c1);
    P.plen[cj] = d2.ord;
    P.netocc[cj] = net;
    P.nbytes[cj] = nbj;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the state above is in LDS
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  int wk = -1;
  if (isw) wk = release_worker<LW>(L, P, s, w);
  woke = rl(wk, 0);
  if (TR3 && lane == 0) TR(r, 18);
  // ------------------------------------------------ outputs, then retire
  o.flush(D, (size_t)(r & (RS - 1)) * PLC);
  finish_slot(D, L, s, r, o, pops, false);
  if (TR3 && lane == 0) {
    TR(r, 29);
    trace_at(D, r, 30, 1ull);  // exe_v finished it
  }
  return true;
}
