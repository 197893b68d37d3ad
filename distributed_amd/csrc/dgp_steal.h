// dgp_steal.h — WorkStealing on MI355X: the cost levels of every processing task
// (steal_time_ratio, /root/reference/distributed/stealing.py:241-277) and one
// balance() call (:401-503), bit-exact with the reference (tests/golden/steal_*.npz).
//
// What makes balance() parallel: worker_objective (scheduler.py:3131-3146) reads the
// plain WorkerState.occupancy, which a balance() never changes (steals are only
// requested; in-flight occupancy is a separate account). So every examined task's
// thief = argmin over the thief set of a key that depends only on (task, worker), and
// the thief set only shrinks. k_best_thief evaluates that argmin for all stealable
// tasks at once against the initial thief set (one wave per task, the thieves spread
// over the lanes). k_balance then walks the bins in the reference's order in one wave:
// acceptance test, in-flight accounts, thief removal, check_idle_saturated. It re-runs
// the argmin (wave-parallel, current thief set) only when the precomputed thief has
// since left the set — exact, because the argmin over a subset that still contains the
// original winner is that winner.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dgp {
namespace steal {

constexpr int N_LEVELS = 15;     // len(WorkStealing.cost_multipliers) (stealing.py:83-85)
constexpr double LATENCY = 0.1;  // stealing.py:37
constexpr int MAXH = 4;          // distinct dependency holders a task's fast thief search handles

struct Prob {
  int W;
  const int32_t* nthreads;
  const double* occ;       // WorkerState.occupancy
  const int32_t* nproc;    // len(ws.processing)
  const int64_t* wnbytes;  // ws.nbytes
  const uint8_t* idle;     // membership of SchedulerState.idle
  const uint8_t* sat;      // membership of SchedulerState.saturated
  double total_occ;
  int64_t total_nthreads;
  int64_t bw;
  int64_t T;
  const int32_t* victim;   // processing_on
  const double* duration;  // get_task_duration
  const uint8_t* fast;     // prefix in fast_tasks
  const int64_t* dep_ptr;
  const int32_t* dep_idx;
  const int64_t* d_nbytes;      // raw nbytes (get_comm_cost)
  const int64_t* d_get_nbytes;  // get_nbytes() (worker_objective, steal_time_ratio)
  const int64_t* h_ptr;         // who_has (CSR)
  const int32_t* h_idx;
  // restrictions of the processing tasks (null: none): valid_workers (scheduler.py
  // :3043-3107) as worker indices (CSR); r_flags bit 0 restricted, bit 1 loose
  const int64_t* r_ptr;
  const int32_t* r_idx;
  const uint8_t* r_flags;
  // the plugin's own state (null: fresh): levels of its stealable bins (key_stealable,
  // stealing.py:220-239; -1 = not in a bin) and the in-flight accounts of steals not yet
  // confirmed (in_flight_occupancy / in_flight_tasks, :191-213)
  const int8_t* level_in;
  const double* ifo_in;
  const int32_t* ift_in;
  uint8_t* checked;  // [W] out: check_idle_saturated ran on this victim (:498-500)
  // work
  int32_t* key;       // [T] level * W + victim, or N_LEVELS * W when not stealable
  int32_t* order;     // [T] task ids sorted by key (stable)
  int32_t* key_sorted;
  int32_t* bin_cnt;   // [N_LEVELS * W + 1]
  int32_t* bin_ptr;   // [N_LEVELS * W + 1] exclusive scan of bin_cnt
  int32_t* s_best;    // [T] per sorted position: thief over the initial thief set
  double* s_cct;      // comm cost to that thief
  double* s_ccv;      // comm cost to the victim
  double* s_dur;      // duration
  // task prep per sorted position: sums of dependency sizes and the distinct holders
  int64_t* s_cget;    // sum of get_nbytes over the dependencies
  int64_t* s_craw;    // sum of raw nbytes
  int32_t* s_nh;      // distinct holders (-1: more than MAXH)
  int32_t* s_hw;      // [T][MAXH] holder worker
  int64_t* s_hg;      // [T][MAXH] get_nbytes it holds
  int64_t* s_hr;      // [T][MAXH] raw nbytes it holds
  // initial thieves sorted by (stack time, ws.nbytes, index), in runs of equal stack time
  uint64_t* tk_a;     // [W] stack-time bits (UINT64_MAX: not a thief)
  int64_t* tk_nb;     // [W]
  int32_t* tk_w;      // [W]
  uint64_t* tk_a2;    // sort scratch
  int64_t* tk_nb2;
  int32_t* tk_w2;
  int32_t* th_order;  // [W] thieves in key order
  int32_t* run_start; // [W + 1]
  double* run_a;      // [W] stack time of each run
  int32_t* run_of_w;  // [W] run of each thief (-1: not a thief)
  int32_t* n_runs;
  int32_t* vs_g;      // [W] victim list (global scratch)
  // outputs
  int8_t* level;
  int32_t *st_task, *st_victim, *st_thief, *st_level;
  double *st_cost, *st_occ_victim, *st_occ_thief;
  long long* n_steals;
  double* inflight_occ;
  int32_t* inflight_tasks;
  uint8_t *idle_out, *sat_out;
};

__device__ __forceinline__ bool holds(const Prob& P, int d, int w) {
  for (int64_t k = P.h_ptr[d]; k < P.h_ptr[d + 1]; k++)
    if (P.h_idx[k] == w) return true;
  return false;
}

// ------------------------------------------------------------------------ levels
// steal_time_ratio -> level (-1: not stealable) and the bin key
__global__ void k_steal_levels(Prob P) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= P.T) return;
  int lv;
  if (P.level_in) {
    lv = P.level_in[t] < N_LEVELS ? P.level_in[t] : -1;  // the bins as the plugin keeps them
  } else if (P.fast[t]) {
    lv = -1;                                       // :252-253
  } else if (P.dep_ptr[t] == P.dep_ptr[t + 1]) {
    lv = 0;                                        // :255-256
  } else {
    const double compute = P.duration[t];
    if (!(compute != 0.0)) {
      lv = -1;                                     // :260-265 long-running
    } else {
      int64_t nb = 0;                              // get_nbytes_deps
      for (int64_t k = P.dep_ptr[t]; k < P.dep_ptr[t + 1]; k++) nb += P.d_get_nbytes[P.dep_idx[k]];
      const double cm = ((double)nb / (double)P.bw + LATENCY) / compute;
      lv = (int)rint(log2(cm) + 6.0);              // int(round(...)): half-even
      if (lv < 1) lv = 1;
      else if (lv >= N_LEVELS) lv = -1;
    }
  }
  P.level[t] = (int8_t)lv;
  const int k = lv >= 0 ? lv * P.W + P.victim[t] : N_LEVELS * P.W;
  P.key[t] = k;
  atomicAdd(&P.bin_cnt[k], 1);
}

// ------------------------------------------------------------------ objective
struct Obj {
  double start;
  int64_t nb;
  int w;
};
__device__ __forceinline__ bool obj_less(const Obj& a, const Obj& b) {
  if (a.start != b.start) return a.start < b.start;
  if (a.nb != b.nb) return a.nb < b.nb;
  return a.w < b.w;
}
__device__ __forceinline__ Obj obj_shfl_xor(const Obj& o, int m) {
  Obj r;
  r.start = __shfl_xor(o.start, m);
  r.nb = __shfl_xor(o.nb, m);
  r.w = __shfl_xor(o.w, m);
  return r;
}

// worker_objective (scheduler.py:3131-3146) of task t on worker w (+ canonical index)
__device__ __forceinline__ Obj objective(const Prob& P, int64_t t, int w) {
  int64_t comm = 0;
  for (int64_t k = P.dep_ptr[t]; k < P.dep_ptr[t + 1]; k++) {
    const int d = P.dep_idx[k];
    if (!holds(P, d, w)) comm += P.d_get_nbytes[d];
  }
  const double stack = P.occ[w] / (double)P.nthreads[w];
  return Obj{stack + (double)comm / (double)P.bw, P.wnbytes[w], w};
}

// get_comm_cost (scheduler.py:3006-3022)
__device__ __forceinline__ double comm_cost(const Prob& P, int64_t t, int w) {
  int64_t nb = 0;
  for (int64_t k = P.dep_ptr[t]; k < P.dep_ptr[t + 1]; k++) {
    const int d = P.dep_idx[k];
    if (!holds(P, d, w)) nb += P.d_nbytes[d];
  }
  return (double)nb / (double)P.bw;
}

// argmin of the objective over the workers with th[w] set (one wave; all lanes return it)
template <class TH>
__device__ __forceinline__ Obj wave_argmin(const Prob& P, int64_t t, TH th) {
  const int lane = threadIdx.x & 63;
  Obj best{INFINITY, INT64_MAX, INT32_MAX};
  for (int w = lane; w < P.W; w += 64) {
    if (!th(w)) continue;
    const Obj o = objective(P, t, w);
    if (obj_less(o, best)) best = o;
  }
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) {
    const Obj o = obj_shfl_xor(best, m);
    if (obj_less(o, best)) best = o;
  }
  return best;
}

// argmin over the valid workers of restricted task t that pass th (one wave)
template <class TH>
__device__ __forceinline__ Obj wave_argmin_valid(const Prob& P, int64_t t, TH th) {
  const int lane = threadIdx.x & 63;
  Obj best{INFINITY, INT64_MAX, INT32_MAX};
  for (int64_t k = P.r_ptr[t] + lane; k < P.r_ptr[t + 1]; k += 64) {
    const int w = P.r_idx[k];
    if (!th(w)) continue;
    const Obj o = objective(P, t, w);
    if (obj_less(o, best)) best = o;
  }
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) {
    const Obj o = obj_shfl_xor(best, m);
    if (obj_less(o, best)) best = o;
  }
  return best;
}
__device__ __forceinline__ bool restricted(const Prob& P, int64_t t) { return P.r_flags && (P.r_flags[t] & 1); }
__device__ __forceinline__ bool loose(const Prob& P, int64_t t) { return P.r_flags && (P.r_flags[t] & 2); }
constexpr int32_t NO_THIEF = -2;  // restricted, not loose, no valid initial thief: never stolen

// one wave per stealable task (sorted position i in [lo, hi)): thief over the initial
// thief set. Rows are independent: ranks can each take a slice (dgp_steal_thief_rows)
// and exchange them (dgp_steal_pack_rows / dgp_steal_unpack_rows).
__global__ void k_best_thief(Prob P, int64_t lo, int64_t hi) {
  const int64_t i = lo + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (i >= hi) return;
  const int64_t t = P.order[i];
  // _get_thief (stealing.py:532-542): potential_thieves & valid_workers when restricted;
  // with no valid thief the loose retry over every thief, or no thief at all
  const bool rs = restricted(P, t);
  Obj b{INFINITY, INT64_MAX, INT32_MAX};
  if (rs) b = wave_argmin_valid(P, t, [&](int w) { return P.idle[w] != 0; });
  if (!rs || (b.w >= P.W && loose(P, t))) b = wave_argmin(P, t, [&](int w) { return P.idle[w] != 0; });
  if ((threadIdx.x & 63) == 0) {
    P.s_best[i] = b.w < P.W ? b.w : (rs ? NO_THIEF : -1);
    P.s_cct[i] = b.w < P.W ? comm_cost(P, t, b.w) : 0.0;
    P.s_ccv[i] = comm_cost(P, t, P.victim[t]);
    P.s_dur[i] = P.duration[t];
    // the task's dependency sizes and distinct holders (for the run-based thief search)
    int64_t cg = 0, cr = 0;
    int nh = 0;
    int hw[MAXH];
    int64_t hg[MAXH], hr[MAXH];
    for (int64_t k = P.dep_ptr[t]; k < P.dep_ptr[t + 1]; k++) {
      const int d = P.dep_idx[k];
      const int64_t g = P.d_get_nbytes[d], rw = P.d_nbytes[d];
      cg += g;
      cr += rw;
      for (int64_t q = P.h_ptr[d]; q < P.h_ptr[d + 1]; q++) {
        const int h = P.h_idx[q];
        int at = -1;
        for (int j = 0; j < MAXH; j++)
          if (j < nh && hw[j] == h) at = j;
        if (at < 0) {
          if (nh >= MAXH) {
            nh = MAXH + 1;
            break;
          }
          at = nh++;
          hw[at] = h;
          hg[at] = 0;
          hr[at] = 0;
        }
        hg[at] += g;
        hr[at] += rw;
      }
      if (nh > MAXH) break;
    }
    P.s_cget[i] = cg;
    P.s_craw[i] = cr;
    P.s_nh[i] = nh > MAXH ? -1 : nh;
    for (int j = 0; j < MAXH; j++) {
      P.s_hw[(size_t)i * MAXH + j] = j < nh && nh <= MAXH ? hw[j] : -1;
      P.s_hg[(size_t)i * MAXH + j] = j < nh && nh <= MAXH ? hg[j] : 0;
      P.s_hr[(size_t)i * MAXH + j] = j < nh && nh <= MAXH ? hr[j] : 0;
    }
  }
}

// One stealable position's k_best_thief output as one 128-byte record: the unit the
// ranks of a sharded balance() exchange (all-gather over RCCL).
struct Row {
  double cct, ccv, dur;
  int64_t cget, craw;
  int32_t best, nh;
  int32_t hw[MAXH];
  int64_t hg[MAXH], hr[MAXH];
};
static_assert(sizeof(Row) == 128, "Row is the exchanged record");

__global__ void k_pack_rows(Prob P, int64_t lo, int64_t hi, Row* out) {
  const int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  Row r;
  r.cct = P.s_cct[i]; r.ccv = P.s_ccv[i]; r.dur = P.s_dur[i];
  r.cget = P.s_cget[i]; r.craw = P.s_craw[i]; r.best = P.s_best[i]; r.nh = P.s_nh[i];
  for (int j = 0; j < MAXH; j++) {
    r.hw[j] = P.s_hw[i * MAXH + j];
    r.hg[j] = P.s_hg[i * MAXH + j];
    r.hr[j] = P.s_hr[i * MAXH + j];
  }
  out[i - lo] = r;
}

__global__ void k_unpack_rows(Prob P, int64_t lo, int64_t hi, const Row* in) {
  const int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  const Row r = in[i - lo];
  P.s_cct[i] = r.cct; P.s_ccv[i] = r.ccv; P.s_dur[i] = r.dur;
  P.s_cget[i] = r.cget; P.s_craw[i] = r.craw; P.s_best[i] = r.best; P.s_nh[i] = r.nh;
  for (int j = 0; j < MAXH; j++) {
    P.s_hw[i * MAXH + j] = r.hw[j];
    P.s_hg[i * MAXH + j] = r.hg[j];
    P.s_hr[i * MAXH + j] = r.hr[j];
  }
}

// ---------------------------------------------------------------- thief order
// sort keys of the initial thieves: stack time (ws.occupancy / nthreads, the first term of
// worker_objective), ws.nbytes, index
__global__ void k_thief_keys(Prob P) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= P.W) return;
  const bool th = P.idle[w] != 0;
  const double a = P.occ[w] / (double)P.nthreads[w];
  P.tk_a[w] = th ? (uint64_t)__double_as_longlong(a) : ~0ull;  // a >= 0: bits order like values
  P.tk_nb[w] = P.wnbytes[w];
  P.tk_w[w] = w;
}
__global__ void k_gather_a(Prob P) {  // stack-time keys in the (nbytes, index) order
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P.W) P.tk_a2[i] = P.tk_a[P.tk_w2[i]];
}
// runs of equal stack time over the sorted thieves (one thread: W steps)
__global__ void k_runs(Prob P) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int r = 0;
  for (int w = 0; w < P.W; w++) P.run_of_w[w] = -1;
  int p = 0;
  for (; p < P.W; p++) {
    const uint64_t a = P.tk_a[p];  // tk_a holds the sorted keys here (see host sequence)
    if (a == ~0ull) break;
    if (p == 0 || a != P.tk_a[p - 1]) {
      P.run_start[r] = p;
      P.run_a[r] = __longlong_as_double((long long)a);
      r++;
    }
    P.run_of_w[P.th_order[p]] = r - 1;
  }
  P.run_start[r] = p;
  *P.n_runs = r;
}

// ---------------------------------------------------------------------- balance
#ifndef DGP_STEAL_WCACHE
#define DGP_STEAL_WCACHE 1  // the thief search's first-window cache (run stack times, ws.nbytes)
#endif
#ifndef DGP_STEAL_PROF
#define DGP_STEAL_PROF 0  // diagnostics: k_balance prints examined / re-evaluated / cycle counts
#endif
__device__ __forceinline__ double rl_f64(double x, int l) {  // lane l's double, via SGPRs
  const long long b = __double_as_longlong(x);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l), hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ int64_t rl_i64s(int64_t x, int l) {  // lane l's int64, via SGPRs
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)x, l), hi = __builtin_amdgcn_readlane((unsigned)(x >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__host__ __device__ inline size_t balance_state_bytes(int W) {
  return (size_t)W * (8 + 8 + 4) + ((size_t)6 * W + 2) * 2 + (size_t)W * 4 + (size_t)W;
}
// One wave; all per-worker balance state in LDS: occupancy, in-flight occupancy, the
// pending task count (len(processing) + in-flight task delta), nthreads, thief / idle /
// saturated flags, the victim list. The walk's accept path reads nothing from global
// memory: on gfx950 loads and stores share one in-order vmcnt, so a global load after the
// request's log stores would wait for those stores too.
__global__ void __launch_bounds__(64) k_balance(Prob P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int W = P.W;
  const int lane = threadIdx.x;
  double* occ = (double*)smem;
  double* ifo = occ + W;
  int32_t* pend = (int32_t*)(ifo + W);      // len(processing) + in_flight_tasks
  // positions, runs and counts below W (<= 4,300 here) fit 16 bits
  uint16_t* run_first = (uint16_t*)(pend + W);  // first possibly-live position of each run
  uint16_t* run_alive = run_first + W;          // live thieves per run
  uint16_t* run_nxt = run_alive + W;            // next run to look at (skips emptied runs)
  uint16_t* nth = run_nxt + W;                  // WorkerState.nthreads
  uint16_t* tho = nth + W;                      // the thieves in key order (th_order)
  uint16_t* rst = tho + W;                      // run_start, R + 1 entries (W + 2 reserved)
  uint8_t* thief = (uint8_t*)(rst + W + 2);
  uint8_t* idle = thief + W;
  uint8_t* sat = idle + W;
  uint8_t* taken = sat + W;                 // topk scratch
  uint8_t* own = taken + W;                 // a window's lane per thief (does a thief repeat in it?)
  int32_t* vs = P.vs_g;                     // victims of the current level (global scratch)
  const int R = *P.n_runs;
  for (int r = lane; r < R; r += 64) {
    run_first[r] = (uint16_t)P.run_start[r];
    run_alive[r] = (uint16_t)(P.run_start[r + 1] - P.run_start[r]);
    run_nxt[r] = (uint16_t)(r + 1);
  }
  for (int r = lane; r <= R; r += 64) rst[r] = (uint16_t)P.run_start[r];
  for (int q = lane; q < P.run_start[R]; q += 64) tho[q] = (uint16_t)P.th_order[q];
  int nth_ = 0, nsat_ = 0;
  for (int w = lane; w < W; w += 64) {
    occ[w] = P.occ[w];
    ifo[w] = P.ifo_in ? P.ifo_in[w] : 0.0;
    pend[w] = P.nproc[w] + (P.ift_in ? P.ift_in[w] : 0);
    nth[w] = (uint16_t)P.nthreads[w];
    P.checked[w] = 0;
    idle[w] = P.idle[w];
    sat[w] = P.sat[w];
    thief[w] = P.idle[w];
    taken[w] = 0;
    nth_ += P.idle[w] != 0;
    nsat_ += P.sat[w] != 0;
  }
  for (int m = 32; m > 0; m >>= 1) {
    nth_ += __shfl_xor(nth_, m);
    nsat_ += __shfl_xor(nsat_, m);
  }
  __syncthreads();
  int n_thieves = nth_;
  long long ns = 0;
  const double avg = P.total_occ / (double)P.total_nthreads;
  auto combined = [&](int w) { return occ[w] + ifo[w]; };                       // :505-506
  auto is_unoccupied = [&](int w, double o, int np) {                           // scheduler.py:2997-3004
    const int nt = nth[w];
    return np < nt || o < nt * avg / 2;
  };
#if DGP_STEAL_PROF
  unsigned long long pr_left = 0, pr_left_cyc = 0, pr_exam = 0, pr_pro = 0, pr_loop = 0, pr_epi = 0, pr_chunks = 0;
  unsigned long long pr_many = 0, pr_win = 0, pr_wcyc = 0;
  const unsigned long long pr_t0 = __builtin_amdgcn_s_memtime();
#endif
  auto finish = [&]() {
    for (int w = lane; w < W; w += 64) {
      P.inflight_occ[w] = ifo[w];
      P.inflight_tasks[w] = pend[w] - P.nproc[w];
      P.idle_out[w] = idle[w];
      P.sat_out[w] = sat[w];
    }
    if (lane == 0) *P.n_steals = ns;
#if DGP_STEAL_PROF
    if (lane == 0)
      printf("k_balance: requests %lld examined %llu thief-left %llu (%llu cycles) total %llu cycles; chunks %llu "
             "prologue %llu loop %llu epilogue %llu; windows with a repeated thief %llu, windows %llu (chain / serial pass %llu cycles)\n", ns, pr_exam,
             pr_left, pr_left_cyc, __builtin_amdgcn_s_memtime() - pr_t0, pr_chunks, pr_pro, pr_loop, pr_epi, pr_many,
             pr_win, pr_wcyc);
#endif
  };
  if (n_thieves == 0 || n_thieves == W) {  // :410-411
    finish();
    return;
  }
  // potential victims (:412-428)
  bool live = false;
  int npv = 0;
  if (nsat_) {
    if (nsat_ >= 20) {
      live = true;
    } else {
      for (int w0 = 0; w0 < W; w0 += 64) {  // ascending index, then stable sort
        const int w = w0 + lane;
        const bool in = w < W && sat[w];
        const unsigned long long m = __ballot(in);
        const int pos = npv + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
        if (in) vs[pos] = w;
        npv += __builtin_popcountll(m);
      }
    }
  } else {  // topk(10, workers, key=combined occupancy): largest first, ties by index
    for (int k = 0; k < 10 && k < W; k++) {
      double bo = -INFINITY;
      int bw_ = INT32_MAX;
      for (int w = lane; w < W; w += 64) {
        if (taken[w]) continue;
        const double o = combined(w);
        if (o > bo || (o == bo && w < bw_)) bo = o, bw_ = w;
      }
      for (int m = 32; m > 0; m >>= 1) {
        const double o2 = __shfl_xor(bo, m);
        const int w2 = __shfl_xor(bw_, m);
        if (o2 > bo || (o2 == bo && w2 < bw_)) bo = o2, bw_ = w2;
      }
      if (bw_ >= W) break;
      if (lane == 0) taken[bw_] = 1;
      __syncthreads();
      if (combined(bw_) > 0.2 && pend[bw_] > (int)nth[bw_] && !thief[bw_]) {
        if (lane == 0) vs[npv] = bw_;
        npv++;
      }
    }
    __syncthreads();
    if (npv == 0) {
      finish();
      return;
    }
  }
  if (!live && lane == 0) {  // sorted(potential_victims, key=combined, reverse=True): stable
    for (int a = 1; a < npv; a++) {
      const int v = vs[a];
      const double o = combined(v);
      int b = a - 1;
      while (b >= 0 && combined(vs[b]) < o) {
        vs[b + 1] = vs[b];
        b--;
      }
      vs[b + 1] = v;
    }
  }
  __syncthreads();
  // the first run at or after r that still has a live thief (emptied runs are skipped
  // through run_nxt, compressed as they are crossed)
  auto find_run = [&](int r) {
    int x = r;
    while (x < R && run_alive[x] == 0) x = run_nxt[x];
    int y = r;
    while (y < R && y != x && run_alive[y] == 0) {
      const int z = run_nxt[y];
      run_nxt[y] = (uint16_t)x;  // every lane writes the same value
      y = z;
    }
    return x;
  };
  // the run stack times from the first live run, one lane each, kept across searches while
  // that start stays (the batch search below reads them by shuffle)
  int wc_r0 = -1;
  double wc_a = 0.0;
  for (int level = 0; level < N_LEVELS; level++) {  // :431
    if (n_thieves == 0) break;
    if (live) {  // list(potential_victims): the saturated set now, ascending index
      npv = 0;
      __syncthreads();
      for (int w0 = 0; w0 < W; w0 += 64) {
        const int w = w0 + lane;
        const bool in = w < W && sat[w];
        const unsigned long long m = __ballot(in);
        const int pos = npv + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
        if (in) vs[pos] = w;
        npv += __builtin_popcountll(m);
      }
      __syncthreads();
    }
    for (int vi = 0; vi < npv; vi++) {  // :434
      const int v = vs[vi];
      const int b0 = P.bin_ptr[level * W + v], b1 = P.bin_ptr[level * W + v + 1];
      if (b0 == b1 || n_thieves == 0) continue;
      // the victim's balance state in registers for its bins (it is never a thief, so only
      // its own requests change it); WorkerState.occupancy is constant in a balance()
      const double occ_v = occ[v];
      double ifo_v = ifo[v];
      int pend_v = pend[v];
      // each chunk's task rows, loaded one chunk ahead (the walk of chunk c hides the loads of c + 1)
      int ntq = 0, nthL = NO_THIEF;
      double ncq = 0.0, nvq = 0.0, ndq = 0.0;
      auto load_rows = [&](int c) {
        const int i = c + lane;
        const bool ok = i < b1;
        ntq = ok ? P.order[i] : 0;
        nthL = ok ? P.s_best[i] : NO_THIEF;  // each lane's task: its precomputed thief
        ncq = ok ? P.s_cct[i] : 0.0;
        nvq = ok ? P.s_ccv[i] : 0.0;
        ndq = ok ? P.s_dur[i] : 0.0;
      };
      load_rows(b0);
      for (int c0 = b0; c0 < b1; c0 += 64) {  // 64 tasks of the bin per load round
#if DGP_STEAL_PROF
        unsigned long long pc0 = __builtin_amdgcn_s_memtime();
        pr_chunks++;
#endif
        const int i = c0 + lane;
        const bool okl = i < b1;
        const int tq = ntq;
        int thL = nthL;
        double cq = ncq;
        const double vq = nvq;
        const double dq = ndq;
        if (c0 + 64 < b1) load_rows(c0 + 64);
        // the thief search's rows of the lane's task, read the first time a search needs them
        bool have_rows = false;
        int nhL = -1;
        int64_t cgL = 0, crL = 0;
        int hwL[MAXH];
        int64_t hgL[MAXH], hrL[MAXH], hnL[MAXH];
        double xL = 0.0;
        double hcL[MAXH];
#pragma unroll
        for (int q = 0; q < MAXH; q++) {
          hwL[q] = 0;
          hgL[q] = hrL[q] = hnL[q] = 0;
          hcL[q] = 0.0;
        }
        auto search_rows = [&]() {
          if (have_rows) return;
          have_rows = true;
          nhL = okl ? P.s_nh[i] : -1;
          cgL = okl ? P.s_cget[i] : 0;
          crL = okl ? P.s_craw[i] : 0;
#pragma unroll
          for (int q = 0; q < MAXH; q++) {
            const bool hj = okl && q < nhL;
            hwL[q] = hj ? P.s_hw[(size_t)i * MAXH + q] : 0;
            hgL[q] = hj ? P.s_hg[(size_t)i * MAXH + q] : 0;
            hrL[q] = hj ? P.s_hr[(size_t)i * MAXH + q] : 0;
          }
#pragma unroll
          for (int q = 0; q < MAXH; q++) hnL[q] = okl && q < nhL ? P.wnbytes[hwL[q]] : 0;
          // the search's comm terms (worker_objective :3136-3138), computed once per task
          xL = (double)cgL / (double)P.bw;
#pragma unroll
          for (int q = 0; q < MAXH; q++) hcL[q] = (double)(cgL - hgL[q]) / (double)P.bw;
        };
        const int nq = min(64, b1 - c0);
        // each lane's thief's balance state, gathered at once (the lanes of one thief hold the
        // same values); LDS holds every thief's accounts as of the last committed window
        bool hasL = thL >= 0;
        int aliveL = hasL && thief[thL] ? 1 : 0;
        double occL = hasL ? occ[thL] : 0.0;
        double ifoL = hasL ? ifo[thL] : 0.0;
        int pendL = hasL ? pend[thL] : 0;
        int ntL = hasL ? (int)nth[thL] : 1;
        // the state-free terms of each task's test and request (the same fp64 operations)
        const double hvL = (vq + dq) / 2;  // (ccv + compute) / 2
        const double dvL = dq + vq;        // compute + ccv
        double dtL = dq + cq;              // compute + cct
        double limL = ntL * avg / 2;        // is_unoccupied's occupancy bound of the thief
        // this chunk's requests (the log entry of move_task_request :498-500): in the lane of
        // the accepted task, written out together
        int accL = 0, thO = 0;
        double ovO = 0.0, otO = 0.0;
        const long long ns0 = ns;
#if DGP_STEAL_PROF
        __builtin_amdgcn_s_waitcnt(0);
        unsigned long long pc1 = __builtin_amdgcn_s_memtime();
        pr_pro += pc1 - pc0;
#endif
        // The walk in windows: from task j up to the next task whose precomputed thief left
        // (d), every task's test and the thief's is_unoccupied run in parallel, each lane with
        // the accounts it would see if every earlier task of the window were accepted; the
        // first rejection, or the task after the first one that fills its thief, ends the
        // accepted prefix [j, b). The victim's in-flight occupancy is one fp64 chain over the
        // window (the reference's order); a thief's accounts are the lane's own unless the
        // thief repeats in the window -- then one serial pass carries them task by task (and
        // replays the accepted prefix if b falls inside). The accepted prefix writes its
        // thieves' accounts to LDS; every lane re-reads its thief's. Task d takes the thief
        // search and runs on its own.
        int j = 0;
        while (j < nq && n_thieves > 0) {
          const bool todo = lane >= j && lane < nq && thL != NO_THIEF;
          const unsigned long long needs = __ballot(todo && !(hasL && aliveL));
          const int d = needs ? (int)__builtin_ctzll(needs) : nq;
          const bool inw = todo && lane < d;
          // which thieves repeat in the window: every lane of the window writes its lane to
          // its thief's slot, a lane that finds another's marks the slot (0xff)
          if (inw) own[thL] = (uint8_t)lane;
          __syncthreads();
          const bool lost_race = inw && own[thL] != (uint8_t)lane;
          __syncthreads();
          if (lost_race) own[thL] = 0xff;
          __syncthreads();
          const bool rep = inw && own[thL] == 0xff;
          const unsigned long long repm = __ballot(rep);
#if DGP_STEAL_PROF
          if (repm) pr_many++;
          const unsigned long long wc0 = __builtin_amdgcn_s_memtime();
#endif
          // the victim's chain over the window; a lane without a thief subtracts +0.0 (exact)
          double vb = 0.0;
          {
            const double dvz = inw ? dvL : 0.0;
            for (int k = j; k < d; k++) {
              vb = lane == k ? ifo_v : vb;
              ifo_v = ifo_v - rl_f64(dvz, k);
            }
          }
          // each task's thief accounts as they would be after the window's earlier tasks:
          // the lane's own unless its thief repeats in the window; then the chain of that
          // thief's tasks (prev = the nearest earlier one) is resolved link by link, all
          // thieves at once (one fp64 add per link, the reference's order)
          double tb = ifoL;
          int pb = pendL;
          unsigned long long mym = 0;  // the window's lanes of this lane's thief when it repeats
          for (unsigned long long rm = repm; rm;) {  // one chain per repeated thief, in task order
            const int k0 = (int)__builtin_ctzll(rm);
            const int x = __builtin_amdgcn_readlane(thL, k0);
            const unsigned long long mx = __ballot(inw && thL == x);
            rm &= ~mx;
            double cur = rl_f64(ifoL, k0);  // every lane of a thief holds its accounts
            const int p0 = __builtin_amdgcn_readlane(pendL, k0);
            for (unsigned long long q = mx; q; q &= q - 1) {
              const int k = (int)__builtin_ctzll(q);
              tb = lane == k ? cur : tb;
              cur = cur + rl_f64(dtL, k);
            }
            if ((mx >> lane) & 1ull) {
              mym = mx;
              pb = p0 + __builtin_popcountll(mx & ((1ull << lane) - 1ull));
            }
          }
#if DGP_STEAL_PROF
          pr_wcyc += __builtin_amdgcn_s_memtime() - wc0;
#endif
          const double ot = occL + tb;          // combined_occupancy of the thief (:505-506)
          const double ov = occ_v + vb;         // ... and of the victim
          const bool acc = ot + cq + dq <= ov - hvL;  // :462-465
          const bool full = acc && !((pb + 1) < ntL || occL + (tb + dtL) < limL);  // :487-493
          const unsigned long long bad = __ballot(inw && !acc), fil = __ballot(inw && full);
          const int fb = bad ? (int)__builtin_ctzll(bad) : 64;
          const int ff = fil ? (int)__builtin_ctzll(fil) : 64;
          const int b = min(min(fb, ff + 1), d);
#if DGP_STEAL_PROF
          pr_exam += __builtin_popcountll(__ballot(inw && lane < b));
          pr_win++;
#endif
          // move_task_request (:279-331) for the accepted prefix
          const bool com = inw && lane < b;
          const unsigned long long cm = __ballot(com);
          if (b < d) ifo_v = rl_f64(vb, b);  // the victim's chain up to the prefix's end
          // the last accepted task of each thief carries its accounts (:327-331)
          const unsigned long long later = mym & ~((2ull << lane) - 1ull) & (b >= 64 ? ~0ull : ((1ull << b) - 1ull));
          if (com && later == 0) {
            ifo[thL] = tb + dtL;
            pend[thL] = pb + 1;
          }
          __syncthreads();
          if (cm && hasL) {
            ifoL = ifo[thL];
            pendL = pend[thL];
          }
          if (com) {
            accL = 1;
            thO = thL;
            ovO = ov;
            otO = ot;
          }
          ns += __builtin_popcountll(cm);
          pend_v -= __builtin_popcountll(cm);
          if (ff < b) {  // task ff filled its thief: no longer a thief (:487-493)
            const int x = __builtin_amdgcn_readlane(thL, ff);
            if (thL == x) aliveL = 0;
            if (lane == 0) {
              thief[x] = 0;
              run_alive[P.run_of_w[x]] -= 1;
            }
            __syncthreads();
            n_thieves--;
          }
          // a rejected task changes nothing (:462-465); one after a fill is tested again
          j = (fb <= ff && b == fb) ? b + 1 : b;
          if (b != d || d >= nq || n_thieves == 0) continue;
          // task d's precomputed thief left (or it had none): every task from d on whose thief
          // left gets a new one now, in parallel (one lane each). _get_thief's argmin reads
          // only the thief set and the plain occupancies (worker_objective :3131-3146), and the
          // set only shrinks, so a winner found now is the winner when the task's turn comes
          // as long as it is still a thief; one that leaves by then is searched again.
#if DGP_STEAL_PROF
          const unsigned long long tp0 = __builtin_amdgcn_s_memtime();
          pr_left++;
#endif
          search_rows();
          const bool sl = lane >= d && lane < nq && thL != NO_THIEF && !(hasL && aliveL);
          // restricted tasks (valid_workers): the plain argmin over their live valid thieves,
          // one task at a time (a loose one with none falls through to the general search)
          bool gen = sl;
          if (P.r_flags) {
            unsigned long long rm = __ballot(sl && restricted(P, tq));
            for (; rm; rm &= rm - 1) {
              const int k = (int)__builtin_ctzll(rm);
              const int tk = __builtin_amdgcn_readlane(tq, k);
              const Obj bo = wave_argmin_valid(P, tk, [&](int w) { return thief[w] != 0; });
              const bool lo_ = loose(P, tk);
              const int nth_k = bo.w < W ? bo.w : (lo_ ? -1 : NO_THIEF);
              const double cc = bo.w < W ? comm_cost(P, tk, bo.w) : 0.0;
              if (lane == k && nth_k != -1) {
                thL = nth_k;
                cq = cc;
                gen = false;
              }
            }
          }
          // many holders (more than MAXH): the plain argmin, one task at a time
          {
            unsigned long long mm = __ballot(gen && nhL < 0);
            for (; mm; mm &= mm - 1) {
              const int k = (int)__builtin_ctzll(mm);
              const int tk = __builtin_amdgcn_readlane(tq, k);
              const Obj bo = wave_argmin(P, tk, [&](int w) { return thief[w] != 0; });
              const double cc = comm_cost(P, tk, bo.w);
              if (lane == k) {
                thL = bo.w;
                cq = cc;
                gen = false;
              }
            }
          }
          // the general search, each lane its own task: the runs of equal stack time in
          // order, each offering its first live non-holder (ordered by (ws.nbytes, index));
          // the first run with one gives the least start, later runs only while their start
          // ties; then the <= MAXH holders with their own comm. ws.nbytes is read only to break
          // a tie of starts.
          {
            const int rf = find_run(0);
            if (!DGP_STEAL_WCACHE || rf != wc_r0) {  // the window of run stack times from rf
              wc_r0 = rf;
              wc_a = rf + lane < R ? P.run_a[rf + lane] : INFINITY;
            }
            int r = rf;
            bool act = gen;
            double bs = INFINITY;   // best start
            int bw_ = INT32_MAX;    // best worker
            int64_t bn = -1;        // its ws.nbytes (-1: not read yet)
            auto nb_of = [&](int w) { return P.wnbytes[w]; };
            while (__ballot(act)) {
              // this lane's run r: its stack time from the window (a shuffle every lane runs)
              const int off = r - wc_r0;
              const bool inw_ = off >= 0 && off < 64;
              double ra = __shfl(wc_a, inw_ ? off : 0);
              if (act) {
                if (!inw_) ra = P.run_a[r];
                const double sv = ra + xL;
                if (bw_ != INT32_MAX && sv > bs) {
                  act = false;
                } else {
                  const int pe = rst[r + 1];
                  int p = run_first[r];
                  while (p < pe && !thief[tho[p]]) p++;
                  run_first[r] = (uint16_t)p;  // the same value from every lane that scans it
                  int q = p;
                  while (q < pe) {
                    const int w = tho[q];
                    bool hold = false;
#pragma unroll
                    for (int jh = 0; jh < MAXH; jh++) hold |= jh < nhL && hwL[jh] == w;
                    if (thief[w] && !hold) break;
                    q++;
                  }
                  if (q < pe) {
                    const int w = tho[q];
                    if (bw_ == INT32_MAX) {
                      bs = sv;
                      bw_ = w;
                    } else if (sv == bs) {  // a tie of starts: ws.nbytes, then the index
                      if (bn < 0) bn = nb_of(bw_);
                      const int64_t nw = nb_of(w);
                      if (nw < bn || (nw == bn && w < bw_)) {
                        bw_ = w;
                        bn = nw;
                      }
                    }
                  }
                  // the next run with a live thief (run_nxt links, compressed as crossed)
                  int x = r + 1;
                  while (x < R && run_alive[x] == 0) x = run_nxt[x];
                  r = x;
                  if (r >= R) act = false;
                }
              }
            }
            if (gen) {
#pragma unroll
              for (int jh = 0; jh < MAXH; jh++) {
                if (jh >= nhL) break;
                const int h = hwL[jh];
                if (!thief[h]) continue;
                const double st = occ[h] / (double)nth[h] + hcL[jh];
                bool better = bw_ == INT32_MAX || st < bs;
                if (!better && st == bs) {
                  if (bn < 0) bn = nb_of(bw_);
                  better = hnL[jh] < bn || (hnL[jh] == bn && h < bw_);
                }
                if (better) {
                  bs = st;
                  bw_ = h;
                  bn = hnL[jh];
                }
              }
              int64_t held_raw = 0;
#pragma unroll
              for (int jh = 0; jh < MAXH; jh++)
                if (jh < nhL && hwL[jh] == bw_) held_raw = hrL[jh];
              thL = bw_ < W ? bw_ : NO_THIEF;
              cq = (double)(crL - held_raw) / (double)P.bw;
            }
          }
          // the searched lanes take their new thief's accounts
          if (sl) {
            hasL = thL >= 0;
            aliveL = hasL ? 1 : 0;
            occL = hasL ? occ[thL] : 0.0;
            ifoL = hasL ? ifo[thL] : 0.0;
            pendL = hasL ? pend[thL] : 0;
            ntL = hasL ? (int)nth[thL] : 1;
            dtL = dq + cq;
            limL = ntL * avg / 2;
          }
#if DGP_STEAL_PROF
          pr_left_cyc += __builtin_amdgcn_s_memtime() - tp0;
#endif
        }
#if DGP_STEAL_PROF
        unsigned long long pc2 = __builtin_amdgcn_s_memtime();
        pr_loop += pc2 - pc1;
#endif
        const unsigned long long am = __ballot(accL != 0);
        if (accL) {
          const long long k = ns0 + __builtin_amdgcn_mbcnt_hi((unsigned)(am >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)am, 0));
          P.st_task[k] = tq;
          P.st_victim[k] = v;
          P.st_thief[k] = thO;
          P.st_level[k] = level;
          P.st_cost[k] = dvL;
          P.st_occ_victim[k] = ovO;
          P.st_occ_thief[k] = otO;
        }
        __syncthreads();
#if DGP_STEAL_PROF
        pr_epi += __builtin_amdgcn_s_memtime() - pc2;
#endif
      }
      if (lane == 0) {
        ifo[v] = ifo_v;
        pend[v] = pend_v;
      }
      __syncthreads();
      // check_idle_saturated(victim, occ=combined) (scheduler.py:2949-2995)
      double o = combined(v);
      if (o < 0) o = occ[v];  // :2974-2975
      const int p = P.nproc[v];
      const int nc = nth[v];
      uint8_t id = 0, sa = 0;
      if (is_unoccupied(v, o, p)) {
        id = 1;
      } else if (p > nc) {
        const double pending = o * (double)(p - nc) / (double)(p * nc);
        if (0.4 < pending && pending > 1.9 * avg) sa = 1;
      }
      if (lane == 0) {
        idle[v] = id;
        sat[v] = sa;
        P.checked[v] = 1;
      }
      __syncthreads();
    }
  }
  finish();
}

// dgp_steal_order's sort helpers: int64 keys as order-preserving uint64, gathers by permutation
__global__ void k_flip_sign(uint64_t* k, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) k[i] ^= 1ull << 63;
}
__global__ void k_gather_u64(const uint64_t* __restrict__ src, const int32_t* __restrict__ perm, uint64_t* dst, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[perm[i]];
}
__global__ void k_gather_i32(const int32_t* __restrict__ src, const int32_t* __restrict__ perm, int32_t* dst, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[perm[i]];
}

inline size_t balance_lds_bytes(int W) { return (balance_state_bytes(W) + 15) & ~(size_t)15; }

}  // namespace steal

__global__ void k_iota32(int32_t* a, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = i;
}
}  // namespace dgp
