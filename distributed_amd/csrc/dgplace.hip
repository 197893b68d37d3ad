// dgplace — MI355X (gfx950) placement engine for the dask.distributed scheduler hot path.
//
// Implements the C ABI of include/dgplace.h. Device-resident state (HBM):
//   * task graph as CSR dependencies + CSR dependents (each dependents row sorted by
//     ascending priority, which is the order _add_to_memory releases a frontier in,
//     /root/reference/distributed/scheduler.py:3298-3307);
//   * per-task replica bitsets who_has[N][ceil(W/64)] (TaskState.who_has, :1275);
//   * per-task state / waiting_on count / waiters count / processing_on;
//   * per-worker occupancy state (WorkerState.task_prefix_count in insertion order,
//     _network_occ, nbytes, len(processing); :406-845) and idle / saturated /
//     idle_task_count membership (SchedulerState.check_idle_saturated, :2949).
//
// A round of the replay (one wave of completions, see tests/golden/gen_golden.py):
//   k_frontier_release   all completions of the round in parallel: atomic decrement of
//                        the dependents' waiting_on counters and the dependencies'
//                        waiters counters; records the position of the completion that
//                        releases each task (the frontier of SchedulerState._add_to_memory)
//   k_candidate_commbytes one wave per newly ready task: OR of its dependencies' replica
//                        bitsets -> candidate workers (decide_worker's candidate union,
//                        :8571-8587) and, per candidate, the exact comm-byte sum of
//                        worker_objective (:3136-3138); HBM-bound gather
//   k_commit             the ordered commit of the round's stimuli (transition engine
//                        order, :2045-2076): completion bookkeeping, releases, frontier
//                        placements (argmin of worker_objective), queue refill
//                        (stimulus_queue_slots_maybe_opened, :4983)
//
// Arithmetic follows CPython's evaluation order of the reference expressions; the
// file is compiled with -ffp-contract=off so no multiply-add is fused.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/dgplace.h"

namespace dgp {

constexpr int PMAX = 8;     // distinct task prefixes held in one worker's task_prefix_count
constexpr int PMAX_G = 64;  // distinct prefixes in SchedulerState._task_prefix_count_global

enum : uint8_t { S_RELEASED = 0, S_WAITING, S_PROCESSING, S_QUEUED, S_NO_WORKER, S_MEMORY };
enum : uint8_t { TF_WANTED = 1, TF_ROOTISH = 2 };
enum : uint8_t { WF_IDLE = 1, WF_SAT = 2, WF_ITC = 4 };
enum : int { ERR_NONE = 0, ERR_PREFIX_CAP = 1, ERR_NO_CANDIDATES = 2, ERR_BAD_STATE = 3, ERR_QUEUE = 4,
             ERR_POOL = 5, ERR_GPREFIX_CAP = 6 };

// device-resident control block (counters and scheduler-global scalars)
struct Ctl {
  unsigned long long n_placed;    // placement log length == next run_id
  unsigned long long n_frontier;  // tasks released by the current round's completions
  unsigned long long pool_used;   // candidate pool entries used by the current round
  long long qhead, qlen;          // SchedulerState.queued (sorted array slice)
  long long n_tasks;              // SchedulerState.n_tasks
  long long n_itc, n_idle, n_sat;  // |idle_task_count|, |idle|, |saturated|
  double g_netocc;                // SchedulerState._network_occ_global
  int g_plen;                     // SchedulerState._task_prefix_count_global (ordered)
  int g_pfx[PMAX_G];
  long long g_pcnt[PMAX_G];
  long long n_unrunnable;
  long long itc_slots;  // sum of _task_slots_available over idle_task_count
  int error;
  int err_task;
};

struct Dev {
  int32_t N, W, WB, P, G;
  int64_t bandwidth, default_data_size;
  double unknown_duration, saturation;
  int32_t sat_inf;
  int64_t total_nthreads;
  // graph (static)
  const int64_t* dep_ptr;
  const int32_t* dep_idx;
  const int64_t* dpt_ptr;
  const int32_t* dpt_idx;
  const int64_t* prio;
  const int32_t* prefix;
  const int32_t* group;
  const uint8_t* tflags;
  const int32_t* order;  // tasks in ascending priority
  // synthetic completion reports
  int64_t* res_nbytes;
  double* res_start;
  double* res_stop;
  // task state
  uint8_t* state;
  int32_t* remaining;  // |waiting_on|
  int32_t* waiters;    // |waiters|
  int32_t* proc_on;    // processing_on (-1 if not processing)
  int64_t* cur_nbytes;
  unsigned long long* holders;  // who_has bitsets [N][WB]
  unsigned long long* ready_key;
  unsigned long long* release_key;
  // candidates of newly ready tasks
  int64_t* cand_off;
  int32_t* cand_n;
  int32_t* pool_w;
  int64_t* pool_comm;
  int64_t pool_cap;
  int32_t* frontier;
  // workers
  int32_t* w_nthreads;
  int32_t* w_cap;
  int32_t* w_nproc;
  int32_t* w_plen;
  int32_t* w_pfx;
  int32_t* w_pcnt;
  int64_t* w_netocc;
  int64_t* w_nbytes;
  uint8_t* w_flags;
  int64_t* w_itcslots;  // this worker's contribution to Ctl::itc_slots
  // tournament tree over idle_task_count keyed (len(processing)/nthreads, worker index)
  int32_t Wp;
  double* t_key;
  int32_t* t_idx;
  // prefixes / groups
  double* pdur;
  double* pmaxexec;
  int64_t* g_size;
  int64_t* g_relwait;
  int64_t* g_left;
  int32_t* g_lastw;
  // queue
  int32_t* qarr;
  // placement log
  int32_t* pl_task;
  int32_t* pl_worker;
  int64_t* pl_comm;
  double* pl_start;
  int64_t* pl_wsnbytes;
  int8_t* pl_route;
  // snapshots
  int64_t snap_cap;
  int32_t* snap_nplaced;
  double* snap_occ;
  int64_t* snap_nbytes;
  int32_t* snap_nproc;
  uint8_t* snap_flags;
  int32_t* snap_nqueued;
  Ctl* ctl;
};

// ------------------------------------------------------------------ device helpers

__device__ __forceinline__ int64_t get_nbytes(const Dev& D, int t) {  // TaskState.get_nbytes :1477
  int64_t v = D.cur_nbytes[t];
  return v >= 0 ? v : D.default_data_size;
}

__device__ __forceinline__ bool holds(const Dev& D, int d, int w) {
  return (D.holders[(size_t)d * D.WB + (w >> 6)] >> (w & 63)) & 1ull;
}

__device__ __forceinline__ void set_error(const Dev& D, int code, int task) {
  if (D.ctl->error == 0) {
    D.ctl->error = code;
    D.ctl->err_task = task;
  }
}

__device__ __forceinline__ double prefix_duration(const Dev& D, int p) {  // _calc_occupancy :1892-1899
  double d = D.pdur[p];
  if (d < 0) {
    if (D.pmaxexec[p] > 0)
      d = 2 * D.pmaxexec[p];
    else
      d = D.unknown_duration;
  }
  return d;
}

__device__ double occupancy(const Dev& D, int w) {  // WorkerState.occupancy :840 -> _calc_occupancy :1884
  double res = 0.0;
  const int n = D.w_plen[w];
  const int* pf = D.w_pfx + (size_t)w * PMAX;
  const int* pc = D.w_pcnt + (size_t)w * PMAX;
  for (int i = 0; i < n; i++) res += prefix_duration(D, pf[i]) * (double)pc[i];
  return res + (double)D.w_netocc[w] / (double)D.bandwidth;
}

__device__ double total_occupancy(const Dev& D) {  // SchedulerState.total_occupancy :1877
  const Ctl* c = D.ctl;
  double res = 0.0;
  for (int i = 0; i < c->g_plen; i++) res += prefix_duration(D, c->g_pfx[i]) * (double)c->g_pcnt[i];
  return res + c->g_netocc / (double)D.bandwidth;
}

// insertion-ordered {prefix: count} dicts with delete-on-zero (:773-784)
__device__ bool wdict_inc(const Dev& D, int w, int p) {
  int* pf = D.w_pfx + (size_t)w * PMAX;
  int* pc = D.w_pcnt + (size_t)w * PMAX;
  int n = D.w_plen[w];
  for (int i = 0; i < n; i++)
    if (pf[i] == p) {
      pc[i]++;
      return true;
    }
  if (n == PMAX) return false;
  pf[n] = p;
  pc[n] = 1;
  D.w_plen[w] = n + 1;
  return true;
}
__device__ void wdict_dec(const Dev& D, int w, int p) {
  int* pf = D.w_pfx + (size_t)w * PMAX;
  int* pc = D.w_pcnt + (size_t)w * PMAX;
  int n = D.w_plen[w];
  for (int i = 0; i < n; i++)
    if (pf[i] == p) {
      if (--pc[i] == 0) {
        for (int k = i + 1; k < n; k++) {
          pf[k - 1] = pf[k];
          pc[k - 1] = pc[k];
        }
        D.w_plen[w] = n - 1;
      }
      return;
    }
}
__device__ bool gdict_inc(const Dev& D, int p) {
  Ctl* c = D.ctl;
  for (int i = 0; i < c->g_plen; i++)
    if (c->g_pfx[i] == p) {
      c->g_pcnt[i]++;
      return true;
    }
  if (c->g_plen == PMAX_G) return false;
  c->g_pfx[c->g_plen] = p;
  c->g_pcnt[c->g_plen] = 1;
  c->g_plen++;
  return true;
}
__device__ void gdict_dec(const Dev& D, int p) {
  Ctl* c = D.ctl;
  for (int i = 0; i < c->g_plen; i++)
    if (c->g_pfx[i] == p) {
      if (--c->g_pcnt[i] == 0) {
        for (int k = i + 1; k < c->g_plen; k++) {
          c->g_pfx[k - 1] = c->g_pfx[k];
          c->g_pcnt[k - 1] = c->g_pcnt[k];
        }
        c->g_plen--;
      }
      return;
    }
}

__device__ __forceinline__ int64_t task_slots_available(const Dev& D, int w) {  // :8762-8767
  return (int64_t)D.w_cap[w] - (int64_t)D.w_nproc[w];  // len(long_running) == 0 in the replay
}
__device__ __forceinline__ bool worker_full(const Dev& D, int w) {  // :8770-8773
  if (D.sat_inf) return false;
  return task_slots_available(D, w) <= 0;
}

__device__ void set_flag(const Dev& D, int w, uint8_t f, bool on, long long* counter) {
  uint8_t fl = D.w_flags[w];
  bool was = (fl & f) != 0;
  if (on && !was) {
    D.w_flags[w] = fl | f;
    (*counter)++;
  } else if (!on && was) {
    D.w_flags[w] = fl & ~f;
    (*counter)--;
  }
}

// argmin over idle_task_count of len(processing)/nthreads, lowest index on ties
// (decide_worker_rootish_queuing_enabled :2230-2233): leaf update + path recombination
__device__ void itc_tree_update(const Dev& D, int w, double key) {
  int pos = D.Wp + w;
  D.t_key[pos] = key;
  D.t_idx[pos] = w;
  double k = key;
  int i = w;
  while (pos > 1) {
    int sib = pos ^ 1;
    double sk = D.t_key[sib];
    int si = D.t_idx[sib];
    bool take_sib = (sk < k) || (sk == k && si < i);
    if (take_sib) {
      k = sk;
      i = si;
    }
    pos >>= 1;
    D.t_key[pos] = k;
    D.t_idx[pos] = i;
  }
}

// SchedulerState.check_idle_saturated :2949-2995 (+ is_unoccupied :2997-3004)
__device__ void check_idle_saturated(const Dev& D, int w) {
  if (D.total_nthreads == 0) return;
  Ctl* c = D.ctl;
  double occ = occupancy(D, w);
  int64_t p = D.w_nproc[w];
  int64_t nt = D.w_nthreads[w];
  set_flag(D, w, WF_SAT, false, &c->n_sat);
  bool unocc = p < nt || occ < (double)nt * (total_occupancy(D) / (double)D.total_nthreads) / 2;
  if (unocc) {
    set_flag(D, w, WF_IDLE, true, &c->n_idle);
  } else {
    set_flag(D, w, WF_IDLE, false, &c->n_idle);
    if (p > nt) {
      double pending = occ * (double)(p - nt) / (double)(p * nt);
      if (0.4 < pending && pending > 1.9 * (total_occupancy(D) / (double)D.total_nthreads))
        set_flag(D, w, WF_SAT, true, &c->n_sat);
    }
  }
  bool itc = !worker_full(D, w);
  set_flag(D, w, WF_ITC, itc, &c->n_itc);
  int64_t contrib = itc ? task_slots_available(D, w) : 0;
  c->itc_slots += contrib - D.w_itcslots[w];
  D.w_itcslots[w] = contrib;
  itc_tree_update(D, w, itc ? (double)D.w_nproc[w] / (double)D.w_nthreads[w] : INFINITY);
}

struct Obj {  // worker_objective tuple (:3131-3146) + canonical worker-index tie-break
  double start;
  int64_t nbytes;
  int32_t w;
};
__device__ __forceinline__ bool obj_less(const Obj& a, const Obj& b) {
  if (a.start != b.start) return a.start < b.start;
  if (a.nbytes != b.nbytes) return a.nbytes < b.nbytes;
  return a.w < b.w;
}
__device__ __forceinline__ Obj objective(const Dev& D, int w, int64_t comm) {
  double stack_time = occupancy(D, w) / (double)D.w_nthreads[w];
  double start_time = stack_time + (double)comm / (double)D.bandwidth;
  return Obj{start_time, D.w_nbytes[w], w};
}
__device__ int64_t comm_bytes(const Dev& D, int t, int w) {  // worker_objective's sum :3136-3138
  int64_t comm = 0;
  for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
    int d = D.dep_idx[k];
    if (!holds(D, d, w)) comm += get_nbytes(D, d);
  }
  return comm;
}

// needs_what[w][d] > 0 <=> some dependent of d (other than `except`) is processing on w
// (w does not hold d here; WorkerState._inc/_dec_needs_replica :800-823)
__device__ bool needed_elsewhere(const Dev& D, int d, int w, int except) {
  for (int64_t k = D.dpt_ptr[d]; k < D.dpt_ptr[d + 1]; k++) {
    int x = D.dpt_idx[k];
    if (x != except && D.proc_on[x] == w) return true;
  }
  return false;
}

// ------------------------------------------------------------ decide_worker paths

__device__ int decide_worker_rootish_queuing_enabled(const Dev& D) {  // :2195-2245
  if (D.ctl->n_itc == 0) return -1;
  return D.t_idx[1];
}

__device__ int decide_worker_rootish_queuing_disabled(const Dev& D, int t) {  // :2135-2193
  bool use_idle = D.ctl->n_idle > 0;
  int gi = D.group[t];
  int w;
  if (D.g_lastw[gi] >= 0 && D.g_left[gi] != 0) {
    w = D.g_lastw[gi];
  } else {
    Obj best{0, 0, -1};
    for (int c = 0; c < D.W; c++) {
      if (use_idle && !(D.w_flags[c] & WF_IDLE)) continue;
      Obj o = objective(D, c, comm_bytes(D, t, c));
      if (best.w < 0 || obj_less(o, best)) best = o;
    }
    if (best.w < 0) return -1;
    w = best.w;
    D.g_left[gi] = (int64_t)floor(((double)D.g_size[gi] / (double)D.total_nthreads) * (double)D.w_nthreads[w]);
  }
  D.g_lastw[gi] = D.g_relwait[gi] > 1 ? w : -1;  // states["released"] + states["waiting"] > 1
  D.g_left[gi] -= 1;
  return w;
}

__device__ int kth_idle(const Dev& D, int64_t k) {
  for (int w = 0; w < D.W; w++)
    if (D.w_flags[w] & WF_IDLE) {
      if (k == 0) return w;
      k--;
    }
  return -1;
}

__device__ int decide_worker_fastpath(const Dev& D) {  // :2283-2305
  bool use_idle = D.ctl->n_idle > 0;
  int64_t n = use_idle ? D.ctl->n_idle : D.W;
  if (n < 20) {
    int best = -1;
    double bocc = 0;
    for (int w = 0; w < D.W; w++) {
      if (use_idle && !(D.w_flags[w] & WF_IDLE)) continue;
      double o = occupancy(D, w);
      if (best < 0 || o < bocc) {
        best = w;
        bocc = o;
      }
    }
    if (bocc == 0) {
      int64_t start = D.ctl->n_tasks % n;
      for (int64_t i = 0; i < n; i++) {
        int c = use_idle ? kth_idle(D, (i + start) % n) : (int)((i + start) % n);
        if (occupancy(D, c) == 0) {
          best = c;
          break;
        }
      }
    }
    return best;
  }
  int64_t k = D.ctl->n_tasks % n;
  return use_idle ? kth_idle(D, k) : (int)k;
}

// decide_worker (:8550-8593) over the candidates precomputed by k_candidate_commbytes
__device__ int decide_worker_candidates(const Dev& D, int t, int64_t* comm_out) {
  int n = D.cand_n[t];
  int64_t off = D.cand_off[t];
  if (n <= 0) {
    set_error(D, ERR_NO_CANDIDATES, t);
    return -1;
  }
  if (n == 1) {
    *comm_out = D.pool_comm[off];
    return D.pool_w[off];
  }
  Obj best = objective(D, D.pool_w[off], D.pool_comm[off]);
  int64_t bcomm = D.pool_comm[off];
  for (int i = 1; i < n; i++) {
    Obj o = objective(D, D.pool_w[off + i], D.pool_comm[off + i]);
    if (obj_less(o, best)) {
      best = o;
      bcomm = D.pool_comm[off + i];
    }
  }
  *comm_out = bcomm;
  return best.w;
}

// ------------------------------------------------------------- commit primitives

// SchedulerState._add_to_processing :3199-3256 (+ WorkerState.add_to_processing :733)
__device__ void add_to_processing(const Dev& D, int t, int w, int8_t route, int64_t comm) {
  Ctl* c = D.ctl;
  if (comm < 0) comm = comm_bytes(D, t, w);
  Obj o = objective(D, w, comm);
  unsigned long long i = c->n_placed++;
  D.pl_task[i] = t;
  D.pl_worker[i] = w;
  D.pl_comm[i] = comm;
  D.pl_start[i] = o.start;
  D.pl_wsnbytes[i] = D.w_nbytes[w];
  D.pl_route[i] = route;
  int p = D.prefix[t];
  if (!wdict_inc(D, w, p)) set_error(D, ERR_PREFIX_CAP, t);
  if (!gdict_inc(D, p)) set_error(D, ERR_GPREFIX_CAP, t);
  D.w_nproc[w]++;
  for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
    int d = D.dep_idx[k];
    if (!holds(D, d, w) && !needed_elsewhere(D, d, w, t)) {
      int64_t nb = get_nbytes(D, d);
      D.w_netocc[w] += nb;
      c->g_netocc += (double)nb;
    }
  }
  D.proc_on[t] = w;
  if (D.state[t] == S_WAITING) D.g_relwait[D.group[t]]--;
  D.state[t] = S_PROCESSING;
  check_idle_saturated(D, w);
  c->n_tasks++;
}

__device__ void queue_insert(const Dev& D, int t) {  // HeapSet.add, kept as a sorted array
  Ctl* c = D.ctl;
  long long lo = c->qhead, hi = c->qhead + c->qlen;
  long long pos = hi;
  int64_t pr = D.prio[t];
  while (pos > lo && D.prio[D.qarr[pos - 1]] > pr) {
    D.qarr[pos] = D.qarr[pos - 1];
    pos--;
  }
  D.qarr[pos] = t;
  c->qlen++;
}

// _transition_waiting_processing :2313-2336 (+ waiting->queued :2761, waiting->no-worker :2772)
__device__ void waiting_processing(const Dev& D, int t) {
  int w;
  int8_t route;
  int64_t comm = -1;
  if (D.tflags[t] & TF_ROOTISH) {
    if (D.sat_inf) {
      route = DGP_ROUTE_ROOTISH_NOQ;
      w = decide_worker_rootish_queuing_disabled(D, t);
    } else {
      route = DGP_ROUTE_ROOTISH_Q;
      w = decide_worker_rootish_queuing_enabled(D);
      if (w < 0) {
        D.state[t] = S_QUEUED;
        D.g_relwait[D.group[t]]--;
        queue_insert(D, t);
        return;
      }
    }
  } else if (D.dep_ptr[t + 1] > D.dep_ptr[t]) {
    route = DGP_ROUTE_NONROOTISH;
    w = decide_worker_candidates(D, t, &comm);
  } else {
    route = DGP_ROUTE_FASTPATH;
    w = decide_worker_fastpath(D);
  }
  if (w < 0) {
    D.state[t] = S_NO_WORKER;
    D.g_relwait[D.group[t]]--;
    D.ctl->n_unrunnable++;
    return;
  }
  add_to_processing(D, t, w, route, comm);
}

// Scheduler.stimulus_queue_slots_maybe_opened :4983-5023 (queued->processing :2797)
__device__ void queue_slots_maybe_opened(const Dev& D) {
  Ctl* c = D.ctl;
  if (c->qlen == 0) return;
  int64_t slots = c->itc_slots;
  for (int64_t k = 0; k < slots; k++) {
    if (c->qlen == 0) return;
    int q = D.qarr[c->qhead];
    int w = decide_worker_rootish_queuing_enabled(D);
    if (w < 0) continue;  // stays queued
    c->qhead++;
    c->qlen--;
    add_to_processing(D, q, w, DGP_ROUTE_ROOTISH_Q, -1);
  }
}

// _transition_memory_released :2444-2505 + remove_all_replicas :3161-3171
__device__ void release_task(const Dev& D, int t) {
  int64_t nb = get_nbytes(D, t);
  unsigned long long* row = D.holders + (size_t)t * D.WB;
  for (int wd = 0; wd < D.WB; wd++) {
    unsigned long long bits = row[wd];
    while (bits) {
      int b = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      D.w_nbytes[wd * 64 + b] -= nb;
    }
    row[wd] = 0;
  }
  D.state[t] = S_RELEASED;
  D.g_relwait[D.group[t]]++;
}

// one completion stimulus (Scheduler.handle_task_finished :5783-5797)
__device__ void completion_stimulus(const Dev& D, int t, unsigned long long key) {
  Ctl* c = D.ctl;
  int w = D.proc_on[t];
  if (w < 0 || D.state[t] != S_PROCESSING) {
    set_error(D, ERR_BAD_STATE, t);
    return;
  }
  // _transition_processing_memory :2366-2442 — TaskPrefix.add_duration EWMA :977-985
  int p = D.prefix[t];
  double duration = D.res_stop[t] - D.res_start[t];
  double old = D.pdur[p];
  D.pdur[p] = old < 0 ? duration : 0.5 * duration + 0.5 * old;
  // set_nbytes (:1480) was applied by k_frontier_release
  // _exit_processing_common -> WorkerState.remove_from_processing :759-771
  D.proc_on[t] = -1;
  wdict_dec(D, w, p);
  gdict_dec(D, p);
  D.w_nproc[w]--;
  for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
    int d = D.dep_idx[k];
    if (!holds(D, d, w) && !needed_elsewhere(D, d, w, t)) {
      int64_t nb = get_nbytes(D, d);
      D.w_netocc[w] -= nb;
      c->g_netocc -= (double)nb;
    }
  }
  check_idle_saturated(D, w);
  // _add_to_memory :3283-3335 — add_replica (the who_has bit was published by
  // k_frontier_release; the replica is new, so ws.nbytes grows by get_nbytes)
  D.w_nbytes[w] += get_nbytes(D, t);
  D.state[t] = S_MEMORY;
  // releases (popped before the frontier: LIFO of the recommendations dict)
  for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
    int d = D.dep_idx[k];
    if (D.release_key[d] == key && D.waiters[d] == 0 && !(D.tflags[d] & TF_WANTED) && D.state[d] == S_MEMORY)
      release_task(D, d);
  }
  if (D.dpt_ptr[t + 1] == D.dpt_ptr[t] && !(D.tflags[t] & TF_WANTED)) release_task(D, t);
  // frontier, ascending priority (dependents rows are pre-sorted)
  for (int64_t k = D.dpt_ptr[t]; k < D.dpt_ptr[t + 1]; k++) {
    int x = D.dpt_idx[k];
    if (D.ready_key[x] == key && D.state[x] == S_WAITING && D.remaining[x] == 0) waiting_processing(D, x);
  }
  queue_slots_maybe_opened(D);
}

// ------------------------------------------------------------------ kernels

// update_graph (:4600-4651): tasks popped in ascending priority; released->waiting
// (:2078-2119) and, when nothing is waited on, straight to processing.
__global__ void k_update_graph(Dev D) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int i = 0; i < D.N; i++) {
    int t = D.order[i];
    D.state[t] = S_WAITING;
    int wo = 0;
    for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
      int d = D.dep_idx[k];
      const unsigned long long* row = D.holders + (size_t)d * D.WB;
      bool any = false;
      for (int wd = 0; wd < D.WB && !any; wd++) any = row[wd] != 0;
      if (!any) wo++;
      if (D.state[d] == S_RELEASED) {
        set_error(D, ERR_BAD_STATE, t);  // priorities must be topological
      } else {
        D.waiters[d]++;
      }
    }
    D.remaining[t] = wo;
    int wt = 0;
    for (int64_t k = D.dpt_ptr[t]; k < D.dpt_ptr[t + 1]; k++) wt += D.state[D.dpt_idx[k]] == S_WAITING;
    D.waiters[t] = wt;
    if (wo == 0) waiting_processing(D, t);
  }
}

// frontier release over the round's completion list L[0..n)
__global__ void k_frontier_release(Dev D, const int32_t* L, int64_t n, unsigned long long round_tag) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    int t = L[j];
    unsigned long long key = round_tag | (unsigned long long)j;
    // the replica this completion creates (who_has / nbytes) is known before the ordered
    // commit: publish it now so k_candidate_commbytes sees it. No stimulus earlier in the
    // round can read it (only t's dependents do, and they become ready at j or later).
    int w = D.proc_on[t];
    if (w >= 0) atomicOr(&D.holders[(size_t)t * D.WB + (w >> 6)], 1ull << (w & 63));
    D.cur_nbytes[t] = D.res_nbytes[t];
    for (int64_t k = D.dpt_ptr[t]; k < D.dpt_ptr[t + 1]; k++) {
      int x = D.dpt_idx[k];
      atomicMax(&D.ready_key[x], key);
      if (atomicSub(&D.remaining[x], 1) == 1) {
        unsigned long long f = atomicAdd(&D.ctl->n_frontier, 1ull);
        D.frontier[f] = x;
      }
    }
    for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
      int d = D.dep_idx[k];
      atomicMax(&D.release_key[d], key);
      atomicSub(&D.waiters[d], 1);
    }
  }
}

// one wave per newly ready task: candidate workers and their comm bytes
__global__ void k_candidate_commbytes(Dev D, int64_t nF) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < nF; i += nwaves) {
    int x = D.frontier[i];
    int64_t d0 = D.dep_ptr[x], d1 = D.dep_ptr[x + 1];
    if (d1 == d0 || (D.tflags[x] & TF_ROOTISH)) {
      if (lane == 0) D.cand_n[x] = 0;
      continue;
    }
    // total dependency bytes
    int64_t tot = 0;
    for (int64_t k = d0 + lane; k < d1; k += 64) tot += get_nbytes(D, D.dep_idx[k]);
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
    // candidate union: OR of replica rows, one bitset word per lane
    int64_t base = 0;
    int total_c = 0;
    // count first
    for (int wd0 = 0; wd0 < D.WB; wd0 += 64) {
      int wd = wd0 + lane;
      unsigned long long acc = 0;
      if (wd < D.WB)
        for (int64_t k = d0; k < d1; k++) acc |= D.holders[(size_t)D.dep_idx[k] * D.WB + wd];
      int cnt = __popcll(acc);
      for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
      total_c += cnt;
    }
    if (lane == 0) {
      base = (int64_t)atomicAdd(&D.ctl->pool_used, (unsigned long long)total_c);
      if (base + total_c > D.pool_cap) set_error(D, ERR_POOL, x);
    }
    base = __shfl(base, 0);
    if (base + total_c > D.pool_cap) continue;
    int64_t pos = base;
    for (int wd0 = 0; wd0 < D.WB; wd0 += 64) {
      int wd = wd0 + lane;
      unsigned long long acc = 0;
      if (wd < D.WB)
        for (int64_t k = d0; k < d1; k++) acc |= D.holders[(size_t)D.dep_idx[k] * D.WB + wd];
      int cnt = __popcll(acc);
      // exclusive prefix over lanes
      int incl = cnt;
      for (int o = 1; o < 64; o <<= 1) {
        int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      int excl = incl - cnt;
      int64_t p = pos + excl;
      while (acc) {
        int b = __ffsll((long long)acc) - 1;
        acc &= acc - 1;
        D.pool_w[p++] = wd * 64 + b;
      }
      pos += __shfl(incl, 63);
    }
    // comm bytes per candidate: total minus the bytes the candidate already holds
    for (int ci = lane; ci < total_c; ci += 64) {
      int c = D.pool_w[base + ci];
      int64_t held = 0;
      for (int64_t k = d0; k < d1; k++) {
        int d = D.dep_idx[k];
        if (holds(D, d, c)) held += get_nbytes(D, d);
      }
      D.pool_comm[base + ci] = tot - held;
    }
    if (lane == 0) {
      D.cand_off[x] = base;
      D.cand_n[x] = total_c;
    }
  }
}

// ordered commit of the round (one thread; the parallel commit replaces this)
__global__ void k_commit(Dev D, const int32_t* L, int64_t n, unsigned long long round_tag) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    for (int64_t j = 0; j < n; j++) {
      completion_stimulus(D, L[j], round_tag | (unsigned long long)j);
      if (D.ctl->error) return;
    }
  }
}

__global__ void k_snapshot(Dev D, int64_t r, int32_t nplaced) {
  if (r >= D.snap_cap) return;
  for (int w = blockIdx.x * blockDim.x + threadIdx.x; w < D.W; w += gridDim.x * blockDim.x) {
    size_t o = (size_t)r * D.W + w;
    D.snap_occ[o] = occupancy(D, w);
    D.snap_nbytes[o] = D.w_nbytes[w];
    D.snap_nproc[o] = D.w_nproc[w];
    D.snap_flags[o] = D.w_flags[w];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    D.snap_nplaced[r] = nplaced;
    D.snap_nqueued[r] = (int32_t)D.ctl->qlen;
  }
}

__global__ void k_init_workers(Dev D) {
  for (int w = blockIdx.x * blockDim.x + threadIdx.x; w < D.W; w += gridDim.x * blockDim.x) {
    D.w_nproc[w] = 0;
    D.w_plen[w] = 0;
    D.w_netocc[w] = 0;
    D.w_nbytes[w] = 0;
    D.w_flags[w] = 0;
    D.w_itcslots[w] = 0;
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 2 * D.Wp; i += gridDim.x * blockDim.x) {
    D.t_key[i] = INFINITY;
    D.t_idx[i] = i < D.Wp ? 0x7fffffff : i - D.Wp;
  }
}

// Scheduler.add_worker (:4418): check_idle_saturated for every new worker, in order
__global__ void k_add_workers(Dev D) {
  if (threadIdx.x == 0 && blockIdx.x == 0)
    for (int w = 0; w < D.W; w++) check_idle_saturated(D, w);
}

}  // namespace dgp

// =================================================================== host side

namespace {

struct Buf {
  void* p = nullptr;
  size_t n = 0;
};

}  // namespace

struct dgp_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  dgp::Dev D{};
  dgp::Ctl* ctl = nullptr;
  std::vector<void*> allocs;
  std::vector<void*> graph_allocs;
  bool have_config = false, have_workers = false, have_graph = false, have_results = false;
  bool graph_done = false;
  int64_t rounds_done = 0;
  int64_t round_start = 0, round_end = 0;  // placement-log slice completed by the next round
  int64_t snap_rounds = 0;
  // host copies
  std::vector<int32_t> nthreads;
  std::vector<double> prefix_defaults;
  std::vector<int64_t> group_sizes;
  int64_t E = 0;
  // timing
  bool timing = false;
  double kms[4] = {0, 0, 0, 0};
  int64_t klaunch[4] = {0, 0, 0, 0};
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> evpool;          // (start, stop) pairs recorded around launches
  std::vector<int> evkind;                 // kernel id per recorded pair
  size_t evused = 0;
  int32_t* d_batch = nullptr;
  int64_t batch_cap = 0;
};

namespace {

int fail(dgp_engine* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  return code;
}

#define HIPCHK(e, call)                                                                       \
  do {                                                                                        \
    hipError_t _st = (call);                                                                  \
    if (_st != hipSuccess)                                                                    \
      return fail(e, DGP_E_HIP, std::string(#call) + ": " + hipGetErrorString(_st));          \
  } while (0)

template <class T>
int dalloc(dgp_engine* e, T** p, size_t count, std::vector<void*>& list) {
  if (count == 0) count = 1;
  hipError_t st = hipMalloc((void**)p, count * sizeof(T));
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(st));
  list.push_back((void*)*p);
  return 0;
}

void free_list(std::vector<void*>& l) {
  for (void* p : l) (void)hipFree(p);
  l.clear();
}

int check_device_error(dgp_engine* e) {
  dgp::Ctl c;
  hipError_t st = hipMemcpyAsync(&c, e->ctl, sizeof c, hipMemcpyDeviceToHost, e->stream);
  if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("sync: ") + hipGetErrorString(st));
  if (c.error) {
    static const char* names[] = {"none", "worker prefix dict overflow (PMAX)", "task without candidates",
                                  "inconsistent task state", "queue", "candidate pool overflow",
                                  "global prefix dict overflow"};
    char buf[160];
    snprintf(buf, sizeof buf, "device engine error %d (%s) at task %d", c.error,
             (c.error >= 0 && c.error <= 6) ? names[c.error] : "?", c.err_task);
    return fail(e, DGP_E_DEVICE, buf);
  }
  return 0;
}

// resolve recorded (start, stop) event pairs into per-kernel totals
int resolve_timing(dgp_engine* e) {
  if (e->evused == 0) return 0;
  HIPCHK(e, hipEventSynchronize(e->evpool[2 * (e->evused - 1) + 1]));
  for (size_t i = 0; i < e->evused; i++) {
    float ms = 0;
    HIPCHK(e, hipEventElapsedTime(&ms, e->evpool[2 * i], e->evpool[2 * i + 1]));
    e->kms[e->evkind[i]] += ms;
  }
  e->evused = 0;
  return 0;
}

template <class F>
int timed_launch(dgp_engine* e, int kid, F&& launch) {
  size_t slot = e->evused;
  if (e->timing) {
    if (slot == (1u << 15)) {
      if (int rc = resolve_timing(e)) return rc;
      slot = 0;
    }
    if (2 * slot + 1 >= e->evpool.size()) {
      hipEvent_t a, b;
      HIPCHK(e, hipEventCreate(&a));
      HIPCHK(e, hipEventCreate(&b));
      e->evpool.push_back(a);
      e->evpool.push_back(b);
      e->evkind.push_back(0);
    }
    e->evkind[slot] = kid;
    HIPCHK(e, hipEventRecord(e->evpool[2 * slot], e->stream));
  }
  launch();
  HIPCHK(e, hipGetLastError());
  if (e->timing) {
    HIPCHK(e, hipEventRecord(e->evpool[2 * slot + 1], e->stream));
    e->evused = slot + 1;
  }
  e->klaunch[kid]++;
  return 0;
}

int read_ctl(dgp_engine* e, dgp::Ctl* c) {
  HIPCHK(e, hipMemcpyAsync(c, e->ctl, sizeof *c, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return 0;
}

int snapshot(dgp_engine* e, int32_t nplaced) {
  if (e->snap_rounds <= 0) return 0;
  int64_t r = e->rounds_done;
  dgp::Dev D = e->D;
  return timed_launch(e, 3, [&] { hipLaunchKernelGGL(dgp::k_snapshot, dim3(8), dim3(256), 0, e->stream, D, r, nplaced); });
}

// one round: completion stimuli for tasks L[0..n) (device pointer), in order
int run_round(dgp_engine* e, const int32_t* dL, int64_t n) {
  dgp::Dev D = e->D;
  HIPCHK(e, hipMemsetAsync(&e->ctl->n_frontier, 0, sizeof(unsigned long long), e->stream));
  HIPCHK(e, hipMemsetAsync(&e->ctl->pool_used, 0, sizeof(unsigned long long), e->stream));
  unsigned long long tag = (unsigned long long)(e->rounds_done + 1) << 32;
  int blocks = (int)std::min<int64_t>((n + 255) / 256, 2048);
  if (blocks < 1) blocks = 1;
  if (int rc = timed_launch(e, 0, [&] {
        hipLaunchKernelGGL(dgp::k_frontier_release, dim3(blocks), dim3(256), 0, e->stream, D, dL, n, tag);
      }))
    return rc;
  dgp::Ctl c;
  if (int rc = read_ctl(e, &c)) return rc;
  int64_t nF = (int64_t)c.n_frontier;
  if (nF > 0) {
    int cb = (int)std::min<int64_t>((nF + 3) / 4, 4096);
    if (int rc = timed_launch(e, 1, [&] {
          hipLaunchKernelGGL(dgp::k_candidate_commbytes, dim3(cb), dim3(256), 0, e->stream, D, nF);
        }))
      return rc;
  }
  unsigned long long before = c.n_placed;
  if (int rc = timed_launch(e, 2, [&] {
        hipLaunchKernelGGL(dgp::k_commit, dim3(1), dim3(64), 0, e->stream, D, dL, n, tag);
      }))
    return rc;
  if (int rc = check_device_error(e)) return rc;
  if (int rc = read_ctl(e, &c)) return rc;
  e->rounds_done++;
  if (int rc = snapshot(e, (int32_t)(c.n_placed - before))) return rc;
  e->round_start = e->round_end;
  e->round_end = (int64_t)c.n_placed;
  return 0;
}

}  // namespace

extern "C" {

int dgp_abi_version(void) { return DGP_ABI_VERSION; }

dgp_engine* dgp_create(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  dgp_engine* e = new dgp_engine();
  e->device = device;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    delete e;
    return nullptr;
  }
  if (hipMalloc((void**)&e->ctl, sizeof(dgp::Ctl)) != hipSuccess) {
    (void)hipStreamDestroy(e->stream);
    delete e;
    return nullptr;
  }
  (void)hipEventCreate(&e->ev0);
  (void)hipEventCreate(&e->ev1);
  e->D.ctl = e->ctl;
  e->D.bandwidth = 100000000;
  e->D.default_data_size = 1024;
  e->D.unknown_duration = 0.5;
  e->D.saturation = 1.1;
  return e;
}

void dgp_destroy(dgp_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  (void)hipStreamSynchronize(e->stream);
  free_list(e->allocs);
  free_list(e->graph_allocs);
  if (e->d_batch) (void)hipFree(e->d_batch);
  (void)hipFree(e->ctl);
  (void)hipEventDestroy(e->ev0);
  (void)hipEventDestroy(e->ev1);
  for (hipEvent_t ev : e->evpool) (void)hipEventDestroy(ev);
  (void)hipStreamDestroy(e->stream);
  delete e;
}

const char* dgp_last_error(const dgp_engine* e) { return e ? e->err.c_str() : "null engine"; }

int dgp_set_config(dgp_engine* e, int64_t bandwidth, int64_t default_data_size, double unknown_duration,
                   double saturation) {
  if (!e) return DGP_E_ARG;
  if (bandwidth <= 0 || default_data_size < 0 || !(saturation > 0))
    return fail(e, DGP_E_ARG, "bandwidth must be > 0, default_data_size >= 0, saturation > 0");
  e->D.bandwidth = bandwidth;
  e->D.default_data_size = default_data_size;
  e->D.unknown_duration = unknown_duration;
  e->D.saturation = saturation;
  e->D.sat_inf = std::isinf(saturation) ? 1 : 0;
  e->have_config = true;
  if (e->have_workers) {  // slot caps depend on the saturation
    std::vector<int32_t> cap(e->nthreads.size());
    for (size_t w = 0; w < cap.size(); w++)
      cap[w] = e->D.sat_inf ? 0 : std::max((int32_t)std::ceil(saturation * e->nthreads[w]), (int32_t)1);
    HIPCHK(e, hipMemcpy(e->D.w_cap, cap.data(), cap.size() * 4, hipMemcpyHostToDevice));
  }
  return 0;
}

int dgp_set_workers(dgp_engine* e, int32_t n_workers, const int32_t* nthreads) {
  if (!e || n_workers <= 0 || !nthreads) return fail(e, DGP_E_ARG, "need n_workers > 0 and nthreads");
  HIPCHK(e, hipSetDevice(e->device));
  if (e->have_workers) return fail(e, DGP_E_STATE, "workers already set");
  e->nthreads.assign(nthreads, nthreads + n_workers);
  dgp::Dev& D = e->D;
  D.W = n_workers;
  D.WB = (n_workers + 63) / 64;
  D.total_nthreads = 0;
  for (int w = 0; w < n_workers; w++) {
    if (nthreads[w] <= 0) return fail(e, DGP_E_ARG, "nthreads must be > 0");
    D.total_nthreads += nthreads[w];
  }
  int rc = 0;
  rc |= dalloc(e, &D.w_nthreads, n_workers, e->allocs);
  rc |= dalloc(e, &D.w_cap, n_workers, e->allocs);
  rc |= dalloc(e, &D.w_nproc, n_workers, e->allocs);
  rc |= dalloc(e, &D.w_plen, n_workers, e->allocs);
  rc |= dalloc(e, &D.w_pfx, (size_t)n_workers * dgp::PMAX, e->allocs);
  rc |= dalloc(e, &D.w_pcnt, (size_t)n_workers * dgp::PMAX, e->allocs);
  rc |= dalloc(e, &D.w_netocc, n_workers, e->allocs);
  rc |= dalloc(e, &D.w_nbytes, n_workers, e->allocs);
  rc |= dalloc(e, &D.w_flags, n_workers, e->allocs);
  rc |= dalloc(e, &D.w_itcslots, n_workers, e->allocs);
  D.Wp = 1;
  while (D.Wp < n_workers) D.Wp <<= 1;
  rc |= dalloc(e, &D.t_key, 2 * (size_t)D.Wp, e->allocs);
  rc |= dalloc(e, &D.t_idx, 2 * (size_t)D.Wp, e->allocs);
  if (rc) return DGP_E_HIP;
  HIPCHK(e, hipMemcpy(D.w_nthreads, nthreads, (size_t)n_workers * 4, hipMemcpyHostToDevice));
  e->have_workers = true;
  return dgp_set_config(e, D.bandwidth, D.default_data_size, D.unknown_duration, D.saturation);
}

int dgp_set_graph(dgp_engine* e, int64_t n_tasks, const int64_t* dep_ptr, const int32_t* dep_idx, const int64_t* prio,
                  const int32_t* prefix_id, int32_t n_prefixes, const double* prefix_default_duration,
                  const int32_t* group_id, int32_t n_groups, const uint8_t* wanted, const int8_t* rootish_override) {
  if (!e) return DGP_E_ARG;
  if (!e->have_workers) return fail(e, DGP_E_STATE, "dgp_set_workers must come first");
  if (n_tasks <= 0 || n_tasks >= (1ll << 31)) return fail(e, DGP_E_ARG, "n_tasks out of range");
  if (n_prefixes <= 0 || n_groups <= 0) return fail(e, DGP_E_ARG, "need prefixes and groups");
  HIPCHK(e, hipSetDevice(e->device));
  free_list(e->graph_allocs);
  const int64_t N = n_tasks;
  const int64_t E = dep_ptr[N];
  if (dep_ptr[0] != 0 || E < 0) return fail(e, DGP_E_ARG, "bad dep_ptr");
  for (int64_t t = 0; t < N; t++)
    if (dep_ptr[t + 1] < dep_ptr[t]) return fail(e, DGP_E_ARG, "dep_ptr not monotone");
  for (int64_t k = 0; k < E; k++)
    if (dep_idx[k] < 0 || dep_idx[k] >= N) return fail(e, DGP_E_ARG, "dep_idx out of range");
  for (int64_t t = 0; t < N; t++) {
    if (prefix_id[t] < 0 || prefix_id[t] >= n_prefixes) return fail(e, DGP_E_ARG, "prefix_id out of range");
    if (group_id[t] < 0 || group_id[t] >= n_groups) return fail(e, DGP_E_ARG, "group_id out of range");
  }
  // dependents CSR, rows sorted by ascending priority
  std::vector<int64_t> dpt_ptr(N + 1, 0);
  for (int64_t k = 0; k < E; k++) dpt_ptr[dep_idx[k] + 1]++;
  for (int64_t t = 0; t < N; t++) dpt_ptr[t + 1] += dpt_ptr[t];
  std::vector<int32_t> dpt_idx(E);
  {
    std::vector<int64_t> fill(dpt_ptr.begin(), dpt_ptr.end() - 1);
    for (int64_t t = 0; t < N; t++)
      for (int64_t k = dep_ptr[t]; k < dep_ptr[t + 1]; k++) dpt_idx[fill[dep_idx[k]]++] = (int32_t)t;
    for (int64_t t = 0; t < N; t++)
      std::sort(dpt_idx.begin() + dpt_ptr[t], dpt_idx.begin() + dpt_ptr[t + 1],
                [&](int32_t a, int32_t b) { return prio[a] < prio[b]; });
  }
  std::vector<int32_t> order(N);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return prio[a] < prio[b]; });
  for (int64_t i = 1; i < N; i++)
    if (prio[order[i]] == prio[order[i - 1]]) return fail(e, DGP_E_ARG, "priorities must be unique");
  for (int64_t t = 0; t < N; t++)
    for (int64_t k = dep_ptr[t]; k < dep_ptr[t + 1]; k++)
      if (prio[dep_idx[k]] >= prio[t]) return fail(e, DGP_E_ARG, "priorities must be topological");
  // static is_rootish per group (:2929-2947); total_nthreads is fixed for the replay
  std::vector<int64_t> gsize(n_groups, 0);
  for (int64_t t = 0; t < N; t++) gsize[group_id[t]]++;
  std::vector<std::vector<int32_t>> gdeps(n_groups);
  for (int64_t t = 0; t < N; t++)
    for (int64_t k = dep_ptr[t]; k < dep_ptr[t + 1]; k++) gdeps[group_id[t]].push_back(group_id[dep_idx[k]]);
  std::vector<uint8_t> grootish(n_groups, 0);
  for (int g = 0; g < n_groups; g++) {
    auto& v = gdeps[g];
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    int64_t sum_len = 0;
    for (int32_t d : v) sum_len += gsize[d];
    grootish[g] = (gsize[g] > e->D.total_nthreads * 2 && (int64_t)v.size() < 5 && sum_len < 5) ? 1 : 0;
  }
  std::vector<uint8_t> tflags(N);
  for (int64_t t = 0; t < N; t++) {
    bool rootish = rootish_override[t] >= 0 ? rootish_override[t] != 0 : grootish[group_id[t]] != 0;
    tflags[t] = (wanted[t] ? dgp::TF_WANTED : 0) | (rootish ? dgp::TF_ROOTISH : 0);
  }
  dgp::Dev& D = e->D;
  D.N = (int32_t)N;
  D.P = n_prefixes;
  D.G = n_groups;
  e->E = E;
  auto& L = e->graph_allocs;
  int rc = 0;
  rc |= dalloc(e, (int64_t**)&D.dep_ptr, N + 1, L);
  rc |= dalloc(e, (int32_t**)&D.dep_idx, E, L);
  rc |= dalloc(e, (int64_t**)&D.dpt_ptr, N + 1, L);
  rc |= dalloc(e, (int32_t**)&D.dpt_idx, E, L);
  rc |= dalloc(e, (int64_t**)&D.prio, N, L);
  rc |= dalloc(e, (int32_t**)&D.prefix, N, L);
  rc |= dalloc(e, (int32_t**)&D.group, N, L);
  rc |= dalloc(e, (uint8_t**)&D.tflags, N, L);
  rc |= dalloc(e, (int32_t**)&D.order, N, L);
  rc |= dalloc(e, &D.res_nbytes, N, L);
  rc |= dalloc(e, &D.res_start, N, L);
  rc |= dalloc(e, &D.res_stop, N, L);
  rc |= dalloc(e, &D.state, N, L);
  rc |= dalloc(e, &D.remaining, N, L);
  rc |= dalloc(e, &D.waiters, N, L);
  rc |= dalloc(e, &D.proc_on, N, L);
  rc |= dalloc(e, &D.cur_nbytes, N, L);
  rc |= dalloc(e, &D.holders, (size_t)N * D.WB, L);
  rc |= dalloc(e, &D.ready_key, N, L);
  rc |= dalloc(e, &D.release_key, N, L);
  rc |= dalloc(e, &D.cand_off, N, L);
  rc |= dalloc(e, &D.cand_n, N, L);
  D.pool_cap = std::max<int64_t>(E + N, 1024);
  rc |= dalloc(e, &D.pool_w, D.pool_cap, L);
  rc |= dalloc(e, &D.pool_comm, D.pool_cap, L);
  rc |= dalloc(e, &D.frontier, N, L);
  rc |= dalloc(e, &D.pdur, n_prefixes, L);
  rc |= dalloc(e, &D.pmaxexec, n_prefixes, L);
  rc |= dalloc(e, &D.g_size, n_groups, L);
  rc |= dalloc(e, &D.g_relwait, n_groups, L);
  rc |= dalloc(e, &D.g_left, n_groups, L);
  rc |= dalloc(e, &D.g_lastw, n_groups, L);
  rc |= dalloc(e, &D.qarr, N, L);
  rc |= dalloc(e, &D.pl_task, N, L);
  rc |= dalloc(e, &D.pl_worker, N, L);
  rc |= dalloc(e, &D.pl_comm, N, L);
  rc |= dalloc(e, &D.pl_start, N, L);
  rc |= dalloc(e, &D.pl_wsnbytes, N, L);
  rc |= dalloc(e, &D.pl_route, N, L);
  if (rc) return DGP_E_HIP;
  auto up = [&](const void* dst, const void* src, size_t bytes) {
    return hipMemcpy(const_cast<void*>(dst), src, bytes, hipMemcpyHostToDevice);
  };
  HIPCHK(e, up(D.dep_ptr, dep_ptr, (N + 1) * 8));
  HIPCHK(e, up(D.dep_idx, dep_idx, std::max<int64_t>(E, 0) * 4));
  HIPCHK(e, up(D.dpt_ptr, dpt_ptr.data(), (N + 1) * 8));
  HIPCHK(e, up(D.dpt_idx, dpt_idx.data(), E * 4));
  HIPCHK(e, up(D.prio, prio, N * 8));
  HIPCHK(e, up(D.prefix, prefix_id, N * 4));
  HIPCHK(e, up(D.group, group_id, N * 4));
  HIPCHK(e, up(D.tflags, tflags.data(), N));
  HIPCHK(e, up(D.order, order.data(), N * 4));
  HIPCHK(e, up(D.g_size, gsize.data(), n_groups * 8));
  e->prefix_defaults.assign(prefix_default_duration, prefix_default_duration + n_prefixes);
  e->group_sizes = gsize;
  e->have_graph = true;
  e->err.clear();
  return dgp_reset(e);
}

int dgp_set_task_results(dgp_engine* e, const int64_t* nbytes, const double* start, const double* stop) {
  if (!e || !e->have_graph) return fail(e, DGP_E_STATE, "graph first");
  HIPCHK(e, hipSetDevice(e->device));
  size_t N = e->D.N;
  HIPCHK(e, hipMemcpy(e->D.res_nbytes, nbytes, N * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(e->D.res_start, start, N * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(e->D.res_stop, stop, N * 8, hipMemcpyHostToDevice));
  e->have_results = true;
  return 0;
}

}  // extern "C"

extern "C" {

int dgp_reset(dgp_engine* e) {
  if (!e || !e->have_graph) return fail(e, DGP_E_STATE, "graph first");
  HIPCHK(e, hipSetDevice(e->device));
  dgp::Dev& D = e->D;
  const size_t N = D.N;
  hipStream_t s = e->stream;
  HIPCHK(e, hipMemsetAsync(e->ctl, 0, sizeof(dgp::Ctl), s));
  HIPCHK(e, hipMemsetAsync(D.state, 0, N, s));
  HIPCHK(e, hipMemsetAsync(D.remaining, 0, N * 4, s));
  HIPCHK(e, hipMemsetAsync(D.waiters, 0, N * 4, s));
  HIPCHK(e, hipMemsetAsync(D.proc_on, 0xff, N * 4, s));
  HIPCHK(e, hipMemsetAsync(D.cur_nbytes, 0xff, N * 8, s));
  HIPCHK(e, hipMemsetAsync(D.holders, 0, N * D.WB * 8, s));
  HIPCHK(e, hipMemsetAsync(D.ready_key, 0, N * 8, s));
  HIPCHK(e, hipMemsetAsync(D.release_key, 0, N * 8, s));
  HIPCHK(e, hipMemsetAsync(D.cand_n, 0, N * 4, s));
  std::vector<double> maxexec(D.P, -1.0);
  HIPCHK(e, hipMemcpyAsync(D.pdur, e->prefix_defaults.data(), D.P * 8, hipMemcpyHostToDevice, s));
  HIPCHK(e, hipMemcpyAsync(D.pmaxexec, maxexec.data(), D.P * 8, hipMemcpyHostToDevice, s));
  HIPCHK(e, hipMemcpyAsync(D.g_relwait, e->group_sizes.data(), D.G * 8, hipMemcpyHostToDevice, s));
  HIPCHK(e, hipMemsetAsync(D.g_left, 0, D.G * 8, s));
  HIPCHK(e, hipMemsetAsync(D.g_lastw, 0xff, D.G * 4, s));
  hipLaunchKernelGGL(dgp::k_init_workers, dim3(8), dim3(256), 0, s, D);
  HIPCHK(e, hipGetLastError());
  hipLaunchKernelGGL(dgp::k_add_workers, dim3(1), dim3(64), 0, s, D);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipStreamSynchronize(s));
  e->graph_done = false;
  e->rounds_done = 0;
  e->round_start = e->round_end = 0;
  e->evused = 0;
  for (int k = 0; k < 4; k++) {
    e->kms[k] = 0;
    e->klaunch[k] = 0;
  }
  return 0;
}

int dgp_update_graph(dgp_engine* e) {
  if (!e || !e->have_graph || !e->have_config) return fail(e, DGP_E_STATE, "config, workers and graph first");
  if (e->graph_done) return fail(e, DGP_E_STATE, "update_graph already ran (dgp_reset first)");
  HIPCHK(e, hipSetDevice(e->device));
  dgp::Dev D = e->D;
  if (int rc = timed_launch(e, 3, [&] { hipLaunchKernelGGL(dgp::k_update_graph, dim3(1), dim3(64), 0, e->stream, D); }))
    return rc;
  if (int rc = check_device_error(e)) return rc;
  dgp::Ctl c;
  if (int rc = read_ctl(e, &c)) return rc;
  e->graph_done = true;
  e->round_start = 0;
  e->round_end = (int64_t)c.n_placed;
  return snapshot(e, (int32_t)c.n_placed);
}

int dgp_run_rounds(dgp_engine* e, int64_t max_rounds, int64_t* n_rounds_out) {
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (!e->have_results) return fail(e, DGP_E_STATE, "dgp_set_task_results first");
  HIPCHK(e, hipSetDevice(e->device));
  int64_t done = 0;
  while (e->round_end > e->round_start && (max_rounds < 0 || done < max_rounds)) {
    if (int rc = run_round(e, e->D.pl_task + e->round_start, e->round_end - e->round_start)) return rc;
    done++;
  }
  if (n_rounds_out) *n_rounds_out = done;
  return 0;
}

int dgp_tasks_finished(dgp_engine* e, int64_t n, const int32_t* tasks, const int64_t* nbytes, const double* start,
                       const double* stop) {
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (n < 0 || (n > 0 && (!tasks || !nbytes || !start || !stop))) return fail(e, DGP_E_ARG, "bad batch");
  if (n == 0) return 0;
  HIPCHK(e, hipSetDevice(e->device));
  if (n > e->batch_cap) {
    if (e->d_batch) (void)hipFree(e->d_batch);
    e->d_batch = nullptr;
    HIPCHK(e, hipMalloc((void**)&e->d_batch, n * 4));
    e->batch_cap = n;
  }
  for (int64_t i = 0; i < n; i++) {
    if (tasks[i] < 0 || tasks[i] >= e->D.N) return fail(e, DGP_E_ARG, "task index out of range");
    int32_t t = tasks[i];
    HIPCHK(e, hipMemcpyAsync(e->D.res_nbytes + t, nbytes + i, 8, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->D.res_start + t, start + i, 8, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->D.res_stop + t, stop + i, 8, hipMemcpyHostToDevice, e->stream));
  }
  HIPCHK(e, hipMemcpyAsync(e->d_batch, tasks, n * 4, hipMemcpyHostToDevice, e->stream));
  return run_round(e, e->d_batch, n);
}

int64_t dgp_num_placements(dgp_engine* e) {
  if (!e) return -1;
  dgp::Ctl c;
  if (read_ctl(e, &c)) return -1;
  return (int64_t)c.n_placed;
}

int dgp_get_placements(dgp_engine* e, int64_t offset, int64_t count, int32_t* task, int32_t* worker,
                       int64_t* comm_bytes, double* start_time, int64_t* ws_nbytes, int8_t* route) {
  if (!e || offset < 0 || count < 0) return fail(e, DGP_E_ARG, "bad range");
  int64_t n = dgp_num_placements(e);
  if (n < 0) return DGP_E_HIP;
  if (offset + count > n) return fail(e, DGP_E_ARG, "range beyond the placement log");
  if (count == 0) return 0;
  const dgp::Dev& D = e->D;
  auto cp = [&](void* dst, const void* src, size_t sz) {
    return dst ? hipMemcpy(dst, (const char*)src + offset * sz, count * sz, hipMemcpyDeviceToHost) : hipSuccess;
  };
  HIPCHK(e, cp(task, D.pl_task, 4));
  HIPCHK(e, cp(worker, D.pl_worker, 4));
  HIPCHK(e, cp(comm_bytes, D.pl_comm, 8));
  HIPCHK(e, cp(start_time, D.pl_start, 8));
  HIPCHK(e, cp(ws_nbytes, D.pl_wsnbytes, 8));
  HIPCHK(e, cp(route, D.pl_route, 1));
  return 0;
}

int dgp_enable_snapshots(dgp_engine* e, int64_t max_rounds) {
  if (!e || !e->have_workers || max_rounds <= 0) return fail(e, DGP_E_ARG, "workers first; max_rounds > 0");
  HIPCHK(e, hipSetDevice(e->device));
  dgp::Dev& D = e->D;
  size_t RW = (size_t)max_rounds * D.W;
  int rc = 0;
  rc |= dalloc(e, &D.snap_nplaced, max_rounds, e->allocs);
  rc |= dalloc(e, &D.snap_occ, RW, e->allocs);
  rc |= dalloc(e, &D.snap_nbytes, RW, e->allocs);
  rc |= dalloc(e, &D.snap_nproc, RW, e->allocs);
  rc |= dalloc(e, &D.snap_flags, RW, e->allocs);
  rc |= dalloc(e, &D.snap_nqueued, max_rounds, e->allocs);
  if (rc) return DGP_E_HIP;
  D.snap_cap = max_rounds;
  e->snap_rounds = max_rounds;
  return 0;
}

int dgp_get_snapshots(dgp_engine* e, int64_t* n_rounds, int32_t* nplaced, double* occupancy, int64_t* ws_nbytes,
                      int32_t* nprocessing, uint8_t* idle, uint8_t* saturated, uint8_t* idle_task_count,
                      int32_t* nqueued) {
  if (!e || e->snap_rounds <= 0) return fail(e, DGP_E_STATE, "snapshots not enabled");
  const dgp::Dev& D = e->D;
  int64_t R = std::min<int64_t>(e->graph_done ? e->rounds_done + 1 : 0, e->snap_rounds);
  if (n_rounds) *n_rounds = R;
  if (R == 0) return 0;
  size_t RW = (size_t)R * D.W;
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (nplaced) HIPCHK(e, hipMemcpy(nplaced, D.snap_nplaced, R * 4, hipMemcpyDeviceToHost));
  if (occupancy) HIPCHK(e, hipMemcpy(occupancy, D.snap_occ, RW * 8, hipMemcpyDeviceToHost));
  if (ws_nbytes) HIPCHK(e, hipMemcpy(ws_nbytes, D.snap_nbytes, RW * 8, hipMemcpyDeviceToHost));
  if (nprocessing) HIPCHK(e, hipMemcpy(nprocessing, D.snap_nproc, RW * 4, hipMemcpyDeviceToHost));
  if (nqueued) HIPCHK(e, hipMemcpy(nqueued, D.snap_nqueued, R * 4, hipMemcpyDeviceToHost));
  std::vector<uint8_t> fl(RW);
  HIPCHK(e, hipMemcpy(fl.data(), D.snap_flags, RW, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < RW; i++) {
    if (idle) idle[i] = (fl[i] & dgp::WF_IDLE) ? 1 : 0;
    if (saturated) saturated[i] = (fl[i] & dgp::WF_SAT) ? 1 : 0;
    if (idle_task_count) idle_task_count[i] = (fl[i] & dgp::WF_ITC) ? 1 : 0;
  }
  return 0;
}

int dgp_get_task_states(dgp_engine* e, uint8_t* state) {
  if (!e || !e->have_graph || !state) return fail(e, DGP_E_ARG, "graph first");
  HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, hipMemcpy(state, e->D.state, e->D.N, hipMemcpyDeviceToHost));
  return 0;
}

int dgp_kernel_times(dgp_engine* e, double* ms, int64_t* launches, int32_t n) {
  if (!e) return DGP_E_ARG;
  if (int rc = resolve_timing(e)) return rc;
  for (int k = 0; k < n && k < 4; k++) {
    if (ms) ms[k] = e->kms[k];
    if (launches) launches[k] = e->klaunch[k];
  }
  return 0;
}

int dgp_set_timing(dgp_engine* e, int enabled) {
  if (!e) return DGP_E_ARG;
  e->timing = enabled != 0;
  return 0;
}

}  // extern "C"
