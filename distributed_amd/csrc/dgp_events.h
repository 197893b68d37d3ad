// dgplace service events: the live scheduler's other placement-input stimuli on the stream
// engine's state between launches. Included by dgplace.hip after dgp_stream.h.
//
// Each kernel is one wave and restates one reference handler's effect on the state that
// placement reads (paths relative to /root/reference/distributed/):
//   k_ev_add_replicas     SchedulerState.add_replica (scheduler.py:3148-3153 ->
//                         WorkerState.add_replica :825-838), from add-keys (:7359-7391)
//   k_ev_remove_replicas  SchedulerState.remove_replica (:3155-3159 -> :786-798), from
//                         release-worker-data (:5807-5815) while another replica remains
//   k_ev_worker_status    handle_worker_status_change (:5850-5883)
//   k_ev_long_running     handle_long_running (:5817-5848)
//   k_ev_heartbeat        heartbeat_worker's TaskPrefix.add_exec_time (:4247-4252, :972-975);
//                         the bandwidth EWMA (:4223-4226) is a host-side Dev field
//   k_ev_worker_flags     idle / saturated membership set by the stealing extension
//                         (stealing.py:396-399, :494-496: check_idle_saturated with the
//                         combined occupancy)
//   k_ev_task_erred       handle_task_erred (:5799-5805) -> stimulus_task_erred (:5094-5127)
//                         -> _transition_processing_erred (:2630-2720) and the cascade it
//                         recommends (waiting -> released -> erred :2579-2605, :2508-2537,
//                         memory -> released :2444-2505)
// Every kernel checks its preconditions before it changes anything and reports a case the
// engine does not model with ERR_UNSUPPORTED (the caller then hands placement back to the
// scheduler): a worker in needs_what scan mode, the last replica going, an erred cascade
// that would cancel processing / waiting work.
#pragma once

namespace dgp {
namespace ev {

using st::lane_id;
using st::NLW;
using st::NXW;
using st::NL_OVF;
using st::SCtl;
using st::nbv;

// An erred task left its dependencies' waiters (:2593-2598) but the stream engine's builder
// counts every completion down on every dependent: a count no completion takes to zero
// keeps it off the frontier when a dependency is recomputed later
constexpr int32_t ERRED_REMAINING = 1 << 30;

__device__ __forceinline__ void ev_init(SCtl& S) {
  if (lane_id() == 0) {
    S.error = 0;
    S.err_task = -1;
    S.stop = 0;
  }
  __syncthreads();
}

// the occupancy check_idle_saturated(ws) reads (WorkerState.occupancy :840-844)
__device__ __forceinline__ void check_idle_saturated(const Dev& D, int w) {  // :2949-2995
  walk_flags(D, w, occupancy(D, w, D.pdur_walk), D.w_nproc[w]);
  itc_check(D, w, false);
}

// del ws.needs_what[d] whatever its count (add_replica :831-834); returns the bytes it
// held in the network occupancy (0 if d was not needed). -1: scan mode (not modelled)
__device__ int64_t needs_drop(const Dev& D, int w, int d, int64_t nb) {
  const int lane = lane_id();
  uint32_t nl = lane < NLW ? D.gw_needs_saved[(size_t)w * NLW + lane] : 0u;
  const uint32_t ctl = st::rlu(nl, NLW - 1);
  if (ctl == NL_OVF) return -1;
  bool found = false;
  const unsigned long long m = st::ballot(lane < NLW - 1 && nl != 0 && (nl >> 8) == (uint32_t)d);
  if (m) {
    if (lane == __builtin_ctzll(m)) nl = 0u;
    found = true;
  } else if ((int)(ctl >> 8) > st::line_used(nl)) {
    uint32_t* X = D.gw_needs_ext + (size_t)w * NXW;
    const uint32_t xe = lane < NXW ? X[lane] : 0u;
    const unsigned long long mx = st::ballot(lane < NXW && xe != 0 && (xe >> 8) == (uint32_t)d);
    if (mx) {
      if (lane == __builtin_ctzll(mx)) X[lane] = 0u;
      found = true;
    }
  }
  if (found && lane == NLW - 1) nl -= 0x100u;
  if (lane < NLW) D.gw_needs_saved[(size_t)w * NLW + lane] = nl;
  __threadfence();
  return found ? nb : 0;
}

__device__ __forceinline__ bool scan_mode(const Dev& D, int w) {
  return D.gw_needs_saved[(size_t)w * NLW + NLW - 1] == NL_OVF;
}

__device__ __forceinline__ int popcount_row(const Dev& D, int t) {
  int n = 0;
  for (int b = 0; b < D.WB; b++) n += __builtin_popcountll(D.holders[(size_t)t * D.WB + b]);
  return n;
}

// SchedulerState.add_replica(ts, ws) for each (task[i], worker[i]) in order
__global__ void __launch_bounds__(64) k_ev_add_replicas(const Dev* __restrict__ Dp, const int32_t* __restrict__ task,
                                                          const int32_t* __restrict__ worker, int n) {
  const Dev& D = *Dp;
  const int lane = lane_id();
  for (int i = 0; i < n; i++) {
    const int t = task[i], w = worker[i];
    if (D.state[t] != S_MEMORY) {  // add_keys only adds replicas of in-memory tasks (:7374-7375)
      if (lane == 0) set_error(D, ERR_BAD_STATE, t);
      return;
    }
    if (holds_any(D, t, w)) continue;  // ts in ws._has_what: nothing (:829-830)
    if (scan_mode(D, w)) {
      if (lane == 0) set_error(D, ERR_UNSUPPORTED, t);
      return;
    }
    const int64_t nb = nbv(D, D.res_nbytes[t]);
    const int64_t freed = needs_drop(D, w, t, nb);
    if (lane == 0) {
      if (freed) {
        D.w_netocc[w] -= freed;
        D.ctl->g_netocc -= (double)freed;
      }
      // the row becomes who_has: it holds the completion's holder already (BLD)
      const int h = D.holder_of[t];
      if (!(D.tdyn[t] & TD_MULTI) && h >= 0) D.holders[(size_t)t * D.WB + (h >> 6)] |= 1ull << (h & 63);
      D.holders[(size_t)t * D.WB + (w >> 6)] |= 1ull << (w & 63);
      D.tdyn[t] |= TD_MULTI;
      D.w_nbytes[w] += nb;
    }
    __threadfence();
    __syncthreads();
  }
}

// SchedulerState.remove_replica(ts, ws) for each (task[i], worker[i]) in order; the last
// replica going (release-worker-data then releases the task: a recompute) is not modelled
__global__ void __launch_bounds__(64) k_ev_remove_replicas(const Dev* __restrict__ Dp, const int32_t* __restrict__ task,
                                                             const int32_t* __restrict__ worker, int n) {
  const Dev& D = *Dp;
  const int lane = lane_id();
  if (lane != 0) return;
  for (int i = 0; i < n; i++) {
    const int t = task[i], w = worker[i];
    if (D.state[t] != S_MEMORY || !holds_any(D, t, w)) {
      set_error(D, ERR_BAD_STATE, t);
      return;
    }
    const bool multi = (D.tdyn[t] & TD_MULTI) != 0;
    if (!multi || popcount_row(D, t) < 2 || scan_mode(D, w)) {
      set_error(D, ERR_UNSUPPORTED, t);
      return;
    }
    D.holders[(size_t)t * D.WB + (w >> 6)] &= ~(1ull << (w & 63));
    D.w_nbytes[w] -= nbv(D, D.res_nbytes[t]);
    if (D.holder_of[t] == w) {  // holder_of names a remaining holder
      for (int b = 0; b < D.WB; b++) {
        const unsigned long long m = D.holders[(size_t)t * D.WB + b];
        if (m) {
          D.holder_of[t] = b * 64 + __builtin_ctzll(m);
          break;
        }
      }
    }
  }
}

// handle_worker_status_change: running -> paused leaves running / idle / idle_task_count /
// saturated (:5879-5883); paused -> running: check_idle_saturated, then
// bulk_schedule_unrunnable_after_adding_worker (no restrictions on this engine: no task is
// no-worker) and the queue refill (:5872-5878). *placed = the placements made.
__global__ void __launch_bounds__(64) k_ev_worker_status(const Dev* __restrict__ Dp, int w, int running,
                                                           long long* placed) {
  const Dev& D = *Dp;
  __shared__ SCtl S;
  ev_init(S);
  const int lane = lane_id();
  if (lane == 0) {
    *placed = 0;
    Ctl* c = D.ctl;
    const uint8_t fl = D.w_flags[w];
    if (!running) {
      if (fl & WF_IDLE) c->n_idle -= 1;
      if (fl & WF_SAT) c->n_sat -= 1;
      if (fl & WF_ITC) {
        c->n_itc -= 1;
        c->itc_slots -= D.w_itcslots[w];
      }
      D.w_itcslots[w] = 0;
      D.w_flags[w] = (uint8_t)((fl & ~(WF_IDLE | WF_SAT | WF_ITC)) | WF_PAUSED);
    } else {
      D.w_flags[w] = (uint8_t)(fl & ~WF_PAUSED);
      check_idle_saturated(D, w);
    }
  }
  __threadfence();
  __syncthreads();
  if (!running) return;
  const long long n = st::refill_queue(D, S);
  if (lane == 0) *placed = n;
}

// handle_long_running: the prefix's duration average takes the compute duration (NaN: None),
// WorkerState.add_to_long_running (prefix counts of the worker and the scheduler, the slot
// _task_slots_available gives back :8765-8767), check_idle_saturated, the queue refill
__global__ void __launch_bounds__(64) k_ev_long_running(const Dev* __restrict__ Dp, int t, double cd,
                                                          long long* placed) {
  const Dev& D = *Dp;
  __shared__ SCtl S;
  ev_init(S);
  const int lane = lane_id();
  const int w = D.proc_on[t];
  if (D.state[t] != S_PROCESSING || w < 0 || w >= D.W || (D.tdyn[t] & TD_LR)) {
    if (lane == 0) set_error(D, ERR_BAD_STATE, t);
    return;
  }
  if (lane == 0) {
    *placed = 0;
    const int p = D.prefix[t];
    if (cd == cd) {  // :5839-5843
      const double old = D.pdur_walk[p];
      const double nd = old < 0 ? cd : (old + cd) / 2;
      D.pdur_walk[p] = D.pdur_cur[p] = D.pdur_pre[p] = nd;
    }
    wdict_dec(D, w, p);  // _remove_from_task_prefix_count :773-784
    gdict_dec(D, p);
    D.tdyn[t] |= TD_LR;
    D.w_cap[w] += 1;
    check_idle_saturated(D, w);
  }
  __threadfence();
  __syncthreads();
  const long long n = st::refill_queue(D, S);
  if (lane == 0) *placed = n;
}

// TaskPrefix.add_exec_time(duration) for each executing task's prefix, in message order
__global__ void k_ev_heartbeat(const Dev* __restrict__ Dp, const int32_t* __restrict__ prefix,
                               const double* __restrict__ duration, int n) {
  const Dev& D = *Dp;
  if (threadIdx.x != 0) return;
  for (int i = 0; i < n; i++) {
    const int p = prefix[i];
    const double d = duration[i];
    const double mx = D.pmaxexec[p];
    D.pmaxexec[p] = d >= mx ? d : mx;  // max(duration, self.max_exec_time)
    if (d > 2 * D.pdur_walk[p]) D.pdur_walk[p] = D.pdur_cur[p] = D.pdur_pre[p] = -1.0;
  }
}

// idle / saturated membership of the given workers as the scheduler holds it
__global__ void k_ev_worker_flags(const Dev* __restrict__ Dp, const int32_t* __restrict__ worker,
                                  const uint8_t* __restrict__ idle, const uint8_t* __restrict__ sat, int n) {
  const Dev& D = *Dp;
  if (threadIdx.x != 0) return;
  Ctl* c = D.ctl;
  for (int i = 0; i < n; i++) {
    const int w = worker[i];
    const uint8_t fl = D.w_flags[w];
    const bool a = idle[i] != 0, b = sat[i] != 0;
    if (a != ((fl & WF_IDLE) != 0)) c->n_idle += a ? 1 : -1;
    if (b != ((fl & WF_SAT) != 0)) c->n_sat += b ? 1 : -1;
    D.w_flags[w] = (uint8_t)((fl & ~(WF_IDLE | WF_SAT)) | (a ? WF_IDLE : 0) | (b ? WF_SAT : 0));
  }
}

// task-erred of processing task t (a current run, no retries left). The closure (t, the
// tasks waiting on it and, transitively, their dependents: none has a replica) errs; every
// dependency outside it loses those waiters and, with none left and no client wanting it,
// is released (memory -> released: remove_all_replicas). A cascade that would release a
// task not in memory (cancel processing / waiting work) is not modelled: the state is put
// back and ERR_UNSUPPORTED reported. Then _exit_processing_common(t) on its worker
// (remove_from_processing, check_idle_saturated, before the releases as in the reference:
// they change ws.nbytes only) and the queue refill of handle_task_erred.
// Scratch: D.frontier (the closure), D.ready (the dependencies that lost a waiter).
__global__ void __launch_bounds__(64) k_ev_task_erred(const Dev* __restrict__ Dp, int t, long long* placed) {
  const Dev& D = *Dp;
  __shared__ SCtl S;
  __shared__ int s_ok;
  ev_init(S);
  const int lane = lane_id();
  const int w = D.proc_on[t];
  if (D.state[t] != S_PROCESSING || w < 0 || w >= D.W) {
    if (lane == 0) set_error(D, ERR_BAD_STATE, t);
    return;
  }
  if (lane == 0) {
    *placed = 0;
    int32_t* Q = D.frontier;
    int32_t* R = D.ready;
    long long qn = 0, rn = 0;
    bool ok = true;
    Q[qn++] = t;
    D.state[t] = S_ERRED;
    for (long long i = 0; i < qn && ok; i++) {  // the closure, marked erred as it is found
      const int x = Q[i];
      for (int64_t k = D.dpt_ptr[x]; k < D.dpt_ptr[x + 1]; k++) {
        const int y = D.dpt_idx[k];
        const uint8_t sy = D.state[y];
        if (sy == S_ERRED || sy == S_MEMORY || (D.tflags[y] & TF_FORGOTTEN)) continue;  // not a dependent any more
        if (sy != S_WAITING) {
          ok = false;
          break;
        }
        D.state[y] = S_ERRED;
        Q[qn++] = y;
      }
    }
    // a member that is a dependency of another member and that nobody else wants: the other
    // member's waiting -> released (:2587-2592) recommends it released, which overrides its
    // "erred" when it is popped later (the dict keeps the place, the value changes), so it
    // ends released or erred by the recommendation dict's order: not restated here
    for (long long i = 1; i < qn && ok; i++) {
      const int y = Q[i];
      for (int64_t k = D.dep_ptr[y]; k < D.dep_ptr[y + 1] && ok; k++) {
        const int d = D.dep_idx[k];
        if (d == t || D.state[d] != S_ERRED || (D.tflags[d] & TF_WANTED)) continue;
        for (long long j = 1; j < qn; j++)
          if (Q[j] == d) {
            ok = false;
            break;
          }
      }
    }
    // waiters.discard for every dependency outside the closure (:2711-2715, :2593-2598)
    const bool dec = ok;
    for (long long i = 0; i < qn && dec; i++) {
      const int x = Q[i];
      for (int64_t k = D.dep_ptr[x]; k < D.dep_ptr[x + 1]; k++) {
        const int d = D.dep_idx[k];
        if (D.state[d] == S_ERRED) continue;
        if (--D.waiters[d] == 0) R[rn++] = d;
      }
    }
    for (long long i = 0; i < rn && ok; i++) {
      const int d = R[i];
      if (!(D.tflags[d] & TF_WANTED) && D.state[d] != S_MEMORY) ok = false;
    }
    if (!ok) {  // put everything back
      for (long long i = 0; i < qn && dec; i++) {
        const int x = Q[i];
        for (int64_t k = D.dep_ptr[x]; k < D.dep_ptr[x + 1]; k++) {
          const int d = D.dep_idx[k];
          if (D.state[d] != S_ERRED) D.waiters[d]++;
        }
      }
      for (long long i = 0; i < qn; i++) D.state[Q[i]] = Q[i] == t ? S_PROCESSING : S_WAITING;
      set_error(D, ERR_UNSUPPORTED, t);
    }
    s_ok = ok ? 1 : 0;
    if (ok) {
      // waiting -> released -> erred for the closure but t (TaskGroup states :1464-1469)
      for (long long i = 1; i < qn; i++) {
        atomicAdd((unsigned long long*)&D.g_relwait[D.group[Q[i]]], (unsigned long long)-1ll);
        D.remaining[Q[i]] = ERRED_REMAINING;  // (see ERRED_REMAINING)
      }
      D.ready_key[0] = (unsigned long long)rn;  // the releases, applied after the worker's part
    }
  }
  __threadfence();
  __syncthreads();
  if (!s_ok) return;
  // _exit_processing_common(t) -> WorkerState.remove_from_processing (:759-771)
  const int p = D.prefix[t];
  const bool lr = (D.tdyn[t] & TD_LR) != 0;
  uint32_t nl = lane < NLW ? D.gw_needs_saved[(size_t)w * NLW + lane] : 0u;
  int64_t freed = 0;
  for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
    const int d = D.dep_idx[k];
    if (holds_any(D, d, w)) continue;
    freed += st::needs_dec(D, S, w, nl, d, nbv(D, D.res_nbytes[d]), t);
  }
  const int npw = D.w_nproc[w] - 1;
  if (npw == 0) st::needs_reset(D, w, nl);
  if (lane < NLW) D.gw_needs_saved[(size_t)w * NLW + lane] = nl;
  __threadfence();
  __syncthreads();
  if (lane == 0) {
    Ctl* c = D.ctl;
    if (lr) {
      D.w_cap[w] -= 1;
      D.tdyn[t] &= (uint8_t)~TD_LR;
    } else {
      wdict_dec(D, w, p);
      gdict_dec(D, p);
    }
    D.w_nproc[w] = npw;
    D.w_netocc[w] -= freed;
    c->g_netocc -= (double)freed;
    D.proc_on[t] = -1;
    check_idle_saturated(D, w);
    // the dependencies nobody waits for: memory -> released (remove_all_replicas :3161-3171)
    const long long rn = (long long)D.ready_key[0];
    for (long long i = 0; i < rn; i++) {
      const int d = D.ready[i];
      if (D.tflags[d] & TF_WANTED) continue;
      const int64_t nb = nbv(D, D.res_nbytes[d]);
      if (D.tdyn[d] & TD_MULTI) {
        for (int b = 0; b < D.WB; b++) {
          unsigned long long m = D.holders[(size_t)d * D.WB + b];
          D.holders[(size_t)d * D.WB + b] = 0;
          for (; m; m &= m - 1) D.w_nbytes[b * 64 + __builtin_ctzll(m)] -= nb;
        }
        D.tdyn[d] &= (uint8_t)~TD_MULTI;
      } else {
        const int hd = D.holder_of[d];
        D.w_nbytes[hd] -= nb;
        D.holders[(size_t)d * D.WB + (hd >> 6)] = 0;
      }
      D.state[d] = S_RELEASED;
      atomicAdd((unsigned long long*)&D.g_relwait[D.group[d]], 1ull);
    }
    if (S.error) set_error(D, S.error, S.err_task);
  }
  __threadfence();
  __syncthreads();
  const long long n = st::refill_queue(D, S);
  if (lane == 0) *placed = n;
}

// ================================================================= worker loss (f2)
// Scheduler.remove_worker (scheduler.py:5180-5303) of a worker with processing tasks or
// sole replicas, decided here instead of by the scheduler. The host passes the worker's
// processing tasks in the order the scheduler iterates ws.processing and its replicas in
// ws.has_what order (the recommendations' order, :5235-5278). Then, as the reference:
//   * the worker leaves running / idle / idle_task_count / saturated (:5226-5231);
//   * remove_replica for each replica (:5270-5271): a task left with none is lost;
//   * recommendations {processing task: released, ..., lost task: released, ...} run
//     through SchedulerState._transitions (:2045-2076): a dict popped LIFO, each
//     transition's recommendations merged with dict.update (a key already present keeps its
//     place). The transitions a loss reaches are restated one by one:
//       processing -> released  _transition_processing_released :2606-2628
//                               (_exit_processing_common :3258-3281, _propagate_released
//                               :3337-3357); -> waiting goes through released (:1961-1984)
//       released -> waiting     _transition_released_waiting :2078-2119
//       memory -> released      _transition_memory_released :2444-2505 (a lost task)
//       waiting -> processing   decide_worker* + _add_to_processing: the update_graph
//                               dispatcher's own (dispatch_prepare / dispatch_collective)
//     A case outside these (a dependency to recompute, a queued or no-worker dependent, a
//     task nobody needs any more) is reported as ERR_UNSUPPORTED; the host checks for them
//     before it calls (dgp_lose_worker), so this is a guard.
// One CTA: lane 0 runs the recommendation machine; a placement takes wave 0 (candidates)
// and, for its collectives, the whole block. Scratch: D.frontier / D.ready = the
// recommendation stack (task, finish), D.ready_key = each task's place in it (-1: absent,
// set by the host before the launch), D.release_key = the tasks marked TD_READD / TD_REWAIT
// (the round engine's key, unused by the stream engine).
enum : int { RC_RELEASED = 0, RC_WAITING = 1, RC_PROCESSING = 2, RC_ERRED = 3 };

// The scheduler's iteration orders the cascade follows where the engine's own (index order)
// differs: row i names task[i] and what it iterates, kind 0 its dependencies
// (_transition_released_waiting :2101, a set), kind 1 its waiters (_transition_memory_released
// :2494 / :2711, a set), kind 2 its dependents (_transition_released_erred :2519, a set);
// rows sorted by (task, kind), checked by the host (dgp_lose_worker_ordered).
enum : int { LO_DEPS = 0, LO_WAITERS = 1, LO_DEPENDENTS = 2 };
struct LossOrder {
  const int32_t* task;
  const int8_t* kind;
  const int64_t* ptr;
  const int32_t* idx;
  int n;
  // the row of (t, k) as [*a, *b) of idx, or false (binary search: a loss names a few tasks)
  __device__ bool row(int t, int k, int64_t* a, int64_t* b) const {
    int lo = 0, hi = n;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (task[m] < t || (task[m] == t && kind[m] < k)) lo = m + 1;
      else hi = m;
    }
    if (lo >= n || task[lo] != t || kind[lo] != k) return false;
    *a = ptr[lo];
    *b = ptr[lo + 1];
    return true;
  }
};

__device__ __forceinline__ void loss_mark(const Dev& D, long long& nmark, int t, uint8_t m) {
  if (!(D.tdyn[t] & (TD_READD | TD_REWAIT))) D.release_key[nmark++] = (unsigned long long)t;
  D.tdyn[t] |= m;
}

__device__ __forceinline__ void rec_push(const Dev& D, long long& sp, int t, int v) {
  long long* at = (long long*)D.ready_key;
  const long long p = at[t];
  if (p >= 0) {  // dict.update on a present key: the value changes, the place stays
    D.ready[p] = v;
    return;
  }
  at[t] = sp;
  D.frontier[sp] = t;
  D.ready[sp] = v;
  sp++;
}

// WorkerState.remove_from_processing (:759-771) of t on its worker x, then (a current
// worker) check_idle_saturated (:3278). needs_what membership is the line's (the removed
// worker's replicas are gone already: TD_WHELD names what it held, for scan mode).
__device__ void loss_exit_processing(const Dev& D, int t, int lost_w, bool tree = true) {
  const int x = D.proc_on[t];
  const int p = D.prefix[t];
  uint32_t* L = D.gw_needs_saved + (size_t)x * SNLW;
  int64_t freed = 0;
  for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
    const int d = D.dep_idx[k];
    if (L[SNLW - 1] == SNL_OVF) {  // scan mode: needed iff not held and nobody else on x needs it
      const bool held = x == lost_w ? (D.tdyn[d] & TD_WHELD) != 0 : holds_any(D, d, x);
      if (!held && !needed_elsewhere(D, d, x, t)) freed += res_nb(D, d);
      continue;
    }
    bool present = false;  // "if dts in self.needs_what" (:770)
    for (int i = 0; i < SNLW - 1 && !present; i++) present = L[i] != 0 && (L[i] >> 8) == (uint32_t)d;
    if (!present && (int)(L[SNLW - 1] >> 8) > 0)
      for (int i = 0; i < SNXW && !present; i++) {
        const uint32_t e = D.gw_needs_ext[(size_t)x * SNXW + i];
        present = e != 0 && (e >> 8) == (uint32_t)d;
      }
    if (present) freed += sneeds_dec(D, x, d, t);
  }
  const int npw = D.w_nproc[x] - 1;
  if (npw == 0) sneeds_reset(D, x);
  if (D.tdyn[t] & TD_LR) {
    D.w_cap[x] -= 1;
    D.tdyn[t] &= (uint8_t)~TD_LR;
  } else {
    wdict_dec(D, x, p);
    gdict_dec(D, p);
  }
  D.w_nproc[x] = npw;
  D.w_netocc[x] -= freed;
  D.ctl->g_netocc -= (double)freed;
  D.proc_on[t] = -1;
  if (x != lost_w) {  // _exit_processing_common: a removed worker is not checked (:3275-3276)
    walk_flags(D, x, occupancy(D, x, D.pdur_walk), D.w_nproc[x]);
    itc_check(D, x, tree);
  }
}

// _transition_released_waiting (:2078-2119) of t: waiting_on = the dependencies without a
// replica; a released dependency is recommended to waiting in turn (:2105-2106: a result lost
// here, or one released earlier -- a recompute chain; either left its own dependencies'
// waiters when it completed, so it is marked TD_READD), every other dependency gains t as a
// waiter when t had left it (TD_READD, :2108-2110). ts.waiters becomes the waiting
// dependents (:2112), recounted for a recomputed task (any other one never left them); a
// dependent still processing counts too: its own processing -> released -> waiting comes
// later in the cascade and adds it then (a task it never left, so the engine does not add
// it again).
__device__ void loss_released_waiting(const Dev& D, const LossOrder& O, long long& sp, long long& nmark, int t) {
  int wo = 0;
  int64_t a = D.dep_ptr[t], b = D.dep_ptr[t + 1];
  const int32_t* row = D.dep_idx;
  if (O.row(t, LO_DEPS, &a, &b)) row = O.idx;  // the scheduler's set order
  const bool readd = (D.tdyn[t] & TD_READD) != 0;
  for (int64_t k = a; k < b; k++) {
    const int d = row[k];
    const uint8_t sd = D.state[d];
    if (sd == S_ERRED || (D.tflags[d] & TF_FORGOTTEN)) {  // a lost / erred dependency
      set_error(D, ERR_UNSUPPORTED, t);
      return;
    }
    bool any = false;
    for (int w = 0; w < D.WB && !any; w++) any = D.holders[(size_t)d * D.WB + w] != 0;
    wo += any ? 0 : 1;
    if (sd == S_RELEASED) {  // recomputed: its recommendation (:2105-2106)
      loss_mark(D, nmark, d, TD_READD);
      rec_push(D, sp, d, RC_WAITING);
      continue;
    }
    if (readd) D.waiters[d] += 1;  // dts.waiters.add(ts) (:2108-2110)
  }
  D.state[t] = S_WAITING;
  D.remaining[t] = wo;
  if (readd) {
    int nw = 0;
    for (int64_t k = D.dpt_ptr[t]; k < D.dpt_ptr[t + 1]; k++) {
      const uint8_t sy = D.state[D.dpt_idx[k]];
      nw += (sy == S_WAITING || sy == S_PROCESSING) ? 1 : 0;
    }
    D.waiters[t] = nw;
  }
  loss_mark(D, nmark, t, TD_REWAIT);
  D.tdyn[t] &= (uint8_t)~TD_READD;
  if (wo == 0) rec_push(D, sp, t, RC_PROCESSING);
}

// dts.waiters.discard(ts) for each dependency of ts that is not erred, and a release
// recommended for one left without waiters and not wanted (:2715-2718, :2593-2598): only a
// dependency in memory is restated (its release frees its replicas)
__device__ bool loss_discard_waiter(const Dev& D, const LossOrder& O, long long& sp, int t) {
  int64_t a = D.dep_ptr[t], b = D.dep_ptr[t + 1];
  const int32_t* row = D.dep_idx;
  if (O.row(t, LO_DEPS, &a, &b)) row = O.idx;
  for (int64_t k = a; k < b; k++) {
    const int d = row[k];
    if (D.state[d] == S_ERRED) continue;  // an erred task has no waiters (:2720)
    if (D.waiters[d] > 0) D.waiters[d] -= 1;
    if (D.waiters[d] == 0 && !(D.tflags[d] & TF_WANTED)) {
      if (D.state[d] != S_MEMORY) {  // the cascade would release a waiting / processing task
        set_error(D, ERR_UNSUPPORTED, d);
        return false;
      }
      rec_push(D, sp, d, RC_RELEASED);
    }
  }
  return true;
}

// Scheduler.remove_worker's KilledWorker (:5239-5265): processing -> erred of t at once, in
// the processing loop (:2630-2720): it leaves the removed worker, its waiters are recommended
// to erred, its dependencies drop it as a waiter
__device__ bool loss_killed(const Dev& D, const LossOrder& O, long long& sp, int t, int lost_w) {
  loss_exit_processing(D, t, lost_w);
  D.state[t] = S_ERRED;
  int64_t a = D.dpt_ptr[t], b = D.dpt_ptr[t + 1];
  const int32_t* row = D.dpt_idx;
  if (O.row(t, LO_WAITERS, &a, &b)) row = O.idx;  // ts.waiters' set order
  for (int64_t k = a; k < b; k++) {
    const int y = row[k];
    const uint8_t sy = D.state[y];
    if (sy == S_WAITING) {
      rec_push(D, sp, y, RC_ERRED);
    } else if (!(sy == S_MEMORY || sy == S_ERRED || sy == S_RELEASED || (D.tflags[y] & TF_FORGOTTEN))) {
      set_error(D, ERR_UNSUPPORTED, y);  // a processing / queued / no-worker dependent
      return false;
    }
  }
  if (!loss_discard_waiter(D, O, sp, t)) return false;
  D.waiters[t] = 0;  // ts.waiters = None
  return true;
}

// client-releases-keys (:5417-5430): the transitions _client_releases_keys' recommendations
// reach (:3400-3419) -- released or forgotten, with every release / forget they recommend in
// turn -- in the order the scheduler runs them, listed by the host (distributed_amd/loss.py
// release_plan restates the recommendation dict LIFO); each applied here by its state now:
//   memory -> released      _transition_memory_released :2444-2505 (remove_all_replicas)
//   processing -> released  _transition_processing_released :2606-2628 (_exit_processing_common
//                           :3258-3281, then _propagate_released :3337-3357)
//   waiting -> released     _transition_waiting_released :2579-2604
//   queued -> released      _transition_queued_released :2784-2795 (queued.remove)
//   no-worker -> released   _transition_no_worker_released :2747-2759 (unrunnable.remove)
//   released                on to forgotten (_propagate_forgotten :3359-3398): the row stays,
//                           released, TF_FORGOTTEN (the host sets the flags)
// A cancelled task leaves its dependencies' waiters (a released one has none). Nothing is
// placed until the queue refill at the end (stimulus_queue_slots_maybe_opened :5430).
__device__ __forceinline__ void cancel_discard(const Dev& D, int t) {
  for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
    const int d = D.dep_idx[k];
    if (D.state[d] != S_RELEASED && D.waiters[d] > 0) D.waiters[d] -= 1;
  }
  D.waiters[t] = 0;  // ts.waiters = None
}

__global__ void __launch_bounds__(64) k_ev_release_tasks(const Dev* __restrict__ Dp, const int32_t* __restrict__ task,
                                                           int n, long long* placed) {
  const Dev& D = *Dp;
  __shared__ SCtl S;
  ev_init(S);
  const int lane = lane_id();
  if (lane == 0) {
    *placed = 0;
    Ctl* c = D.ctl;
    for (int i = 0; i < n && c->error == 0; i++) {
      const int t = task[i];
      const uint8_t st = D.state[t];
      if (st == S_RELEASED) continue;  // on to forgotten: the flag only
      if (st == S_MEMORY) {
        const int64_t nb = nbv(D, D.res_nbytes[t]);
        for (int b = 0; b < D.WB; b++) {
          unsigned long long m = D.holders[(size_t)t * D.WB + b];
          D.holders[(size_t)t * D.WB + b] = 0;
          for (; m; m &= m - 1) D.w_nbytes[b * 64 + __builtin_ctzll(m)] -= nb;
        }
        D.tdyn[t] &= (uint8_t)~TD_MULTI;
        D.holder_of[t] = -1;
      } else if (st == S_PROCESSING) {
        loss_exit_processing(D, t, -1, false);
        D.holder_of[t] = -1;
        cancel_discard(D, t);
      } else if (st == S_WAITING) {
        cancel_discard(D, t);
        // waiting_on = None: no later completion of a dependency makes it runnable (the
        // builder counts completions down on every dependent)
        D.remaining[t] = ERRED_REMAINING;
      } else if (st == S_QUEUED) {
        long long q = c->qhead;
        const long long e = c->qhead + c->qlen;
        while (q < e && D.qarr[q] != t) q++;
        if (q == e) {
          set_error(D, ERR_BAD_STATE, t);
          break;
        }
        for (; q + 1 < e; q++) D.qarr[q] = D.qarr[q + 1];
        c->qlen -= 1;
        cancel_discard(D, t);
      } else if (st == S_NO_WORKER) {
        c->n_unrunnable--;
        cancel_discard(D, t);
      } else {
        set_error(D, ERR_UNSUPPORTED, t);
        break;
      }
      if (st != S_WAITING) atomicAdd((unsigned long long*)&D.g_relwait[D.group[t]], 1ull);  // released + waiting
      D.state[t] = S_RELEASED;
    }
    if (S.error) set_error(D, S.error, S.err_task);
  }
  __threadfence();
  __syncthreads();
  if (D.ctl->error) return;
  const long long m = st::refill_queue(D, S);
  if (lane == 0) *placed = m;
}

// lane 0: pop recommendations until one is a placement (returns its task) or none is left
// (-1). ERR_UNSUPPORTED stops the machine.
__device__ int loss_machine(const Dev& D, const LossOrder& O, long long& sp, long long& nmark, int lost_w) {
  long long* at = (long long*)D.ready_key;
  while (sp > 0 && D.ctl->error == 0) {
    sp--;
    const int t = D.frontier[sp];
    const int v = D.ready[sp];
    at[t] = -1;
    const uint8_t st = D.state[t];
    if ((v == RC_RELEASED && st == S_RELEASED) || (v == RC_WAITING && st == S_WAITING) ||
        (v == RC_PROCESSING && st == S_PROCESSING) || (v == RC_ERRED && st == S_ERRED))
      continue;  // start == finish (:1936-1937)
    if (st == S_WAITING && v == RC_ERRED) {
      // waiting -> released (:2579-2605: its dependencies drop it; exception_blame is set, so
      // no recommendation for itself and ts.waiters = None), then released -> erred
      // (:2507-2537: every dependent without a replica is recommended to erred)
      if (!loss_discard_waiter(D, O, sp, t)) break;
      D.waiters[t] = 0;
      D.remaining[t] = ERRED_REMAINING;
      D.state[t] = S_ERRED;
      atomicAdd((unsigned long long*)&D.g_relwait[D.group[t]], (unsigned long long)-1ll);
      int64_t a = D.dpt_ptr[t], b = D.dpt_ptr[t + 1];
      const int32_t* row = D.dpt_idx;
      if (O.row(t, LO_DEPENDENTS, &a, &b)) row = O.idx;  // ts.dependents' set order
      for (int64_t k = a; k < b; k++) {
        const int y = row[k];
        bool held = false;
        for (int w = 0; w < D.WB && !held; w++) held = D.holders[(size_t)y * D.WB + w] != 0;
        if (!held && !(D.tflags[y] & TF_FORGOTTEN)) rec_push(D, sp, y, RC_ERRED);
      }
      continue;
    }
    const bool needed = D.waiters[t] > 0 || (D.tflags[t] & TF_WANTED);
    if (st == S_PROCESSING && (v == RC_RELEASED || v == RC_WAITING)) {
      loss_exit_processing(D, t, lost_w);
      D.state[t] = S_RELEASED;
      atomicAdd((unsigned long long*)&D.g_relwait[D.group[t]], 1ull);
      if (!needed) {  // _propagate_released would release its dependencies (:3346-3353)
        set_error(D, ERR_UNSUPPORTED, t);
        break;
      }
      rec_push(D, sp, t, RC_WAITING);  // :3343-3344
      if (v == RC_WAITING) loss_released_waiting(D, O, sp, nmark, t);  // through released (:1961-1984)
      continue;
    }
    if (st == S_RELEASED && v == RC_WAITING) {
      loss_released_waiting(D, O, sp, nmark, t);
      continue;
    }
    if (st == S_NO_WORKER && v == RC_WAITING) {  // through released: _transition_no_worker_released :2747-2759
      D.ctl->n_unrunnable--;  // unrunnable.remove
      D.state[t] = S_RELEASED;
      atomicAdd((unsigned long long*)&D.g_relwait[D.group[t]], 1ull);
      if (!needed) {  // _propagate_released would release its dependencies (:3346-3353)
        set_error(D, ERR_UNSUPPORTED, t);
        break;
      }
      rec_push(D, sp, t, RC_WAITING);
      loss_released_waiting(D, O, sp, nmark, t);
      continue;
    }
    if (st == S_MEMORY && v == RC_RELEASED) {  // :2444-2505: a lost result, or a release
      // remove_all_replicas (:2475): the holders left (none for a lost result)
      for (int w = 0; w < D.WB; w++) {
        unsigned long long m = D.holders[(size_t)t * D.WB + w];
        D.holders[(size_t)t * D.WB + w] = 0;
        for (; m; m &= m - 1) D.w_nbytes[w * 64 + __builtin_ctzll(m)] -= res_nb(D, t);
      }
      D.tdyn[t] &= (uint8_t)~TD_MULTI;
      D.state[t] = S_RELEASED;
      D.holder_of[t] = -1;
      atomicAdd((unsigned long long*)&D.g_relwait[D.group[t]], 1ull);
      if (needed) {
        rec_push(D, sp, t, RC_WAITING);
        loss_mark(D, nmark, t, TD_READD);
      }
      int64_t a = D.dpt_ptr[t], b = D.dpt_ptr[t + 1];
      const int32_t* row = D.dpt_idx;
      if (O.row(t, LO_WAITERS, &a, &b)) row = O.idx;  // the scheduler's set order of ts.waiters
      if (D.waiters[t] == 0) b = a;                   // ts.waiters is empty
      for (int64_t k = a; k < b; k++) {  // its waiters (:2494-2500)
        const int y = row[k];
        const uint8_t sy = D.state[y];
        if (sy == S_PROCESSING) {
          rec_push(D, sp, y, RC_WAITING);
        } else if (sy == S_WAITING) {
          if (!(D.tdyn[y] & TD_REWAIT)) D.remaining[y] += 1;  // waiting_on.add (a set)
        } else if (sy == S_NO_WORKER) {
          rec_push(D, sp, y, RC_WAITING);
        } else if (sy == S_QUEUED) {
          // stays queued (:2494-2500 names neither) but no longer in ts.waiters once t is
          // re-waited, while its completion would still count down the engine's count
          set_error(D, ERR_UNSUPPORTED, y);
          break;
        }
      }
      continue;
    }
    if (st == S_WAITING && v == RC_PROCESSING) return t;  // decide_worker + _add_to_processing
    set_error(D, ERR_UNSUPPORTED, t);
  }
  return -1;
}

// mode LM_LOSS: Scheduler.remove_worker of w (proc: its processing tasks, recommended released).
// LM_GRAPH (w < 0): a later graph's update_graph stimulus whose tasks recompute released
// earlier dependencies (:4598-4611, dgp_graph_stimulus): proc = the runnable new tasks in the
// recommendation dict's order, each recommended waiting (none is in a waiters set yet: TD_READD).
// LM_RELEASE (w < 0): Scheduler._reschedule (:7900-7924): transitions({key: "released"}) of
// each processing task in proc
enum : int { LM_LOSS = 0, LM_GRAPH = 1, LM_RELEASE = 2 };
__global__ void __launch_bounds__(CTA) k_ev_lose_worker(const Dev* __restrict__ Dp, int mode, int w,
                                                        const int32_t* __restrict__ proc,
                                                        int n_proc, const int8_t* __restrict__ killed,
                                                        const int32_t* __restrict__ held, int n_held, LossOrder O,
                                                        long long* placed) {
  __shared__ Dev s_dev;  // Dev and Ctl in LDS, as the update_graph dispatcher works on them
  __shared__ Ctl s_ctl;
  {
    const uint32_t* sd = (const uint32_t*)Dp;
    const uint32_t* sc = (const uint32_t*)Dp->ctl;
    for (int i = threadIdx.x; i < (int)(sizeof(Dev) / 4); i += blockDim.x) ((uint32_t*)&s_dev)[i] = sd[i];
    for (int i = threadIdx.x; i < (int)(sizeof(Ctl) / 4); i += blockDim.x) ((uint32_t*)&s_ctl)[i] = sc[i];
    __syncthreads();
    if (threadIdx.x == 0) s_dev.ctl = &s_ctl;
    __syncthreads();
  }
  Ctl* const ctl_g = Dp->ctl;
  const Dev& D = s_dev;
  Ctl* c = D.ctl;
  __shared__ CoopShared S;
  __shared__ long long s_sp, s_nmark;
  __shared__ int s_x;
  const int64_t pl0 = (int64_t)c->n_placed;
  const double* dur = D.pdur_cur;
  if (threadIdx.x == 0 && mode == LM_LOSS) {
    // the worker table part (:5226-5231): out of running / idle / idle_task_count / saturated
    D.w_flags[w] |= WF_PAUSED;
    walk_flags(D, w, occupancy(D, w, D.pdur_walk), D.w_nproc[w]);
    itc_check(D, w, false);
    // remove_replica for every replica the worker holds (:5270-5271), in has_what order
    for (int i = 0; i < n_held; i++) {
      const int t = held[i];
      unsigned long long* row = D.holders + (size_t)t * D.WB;
      row[w >> 6] &= ~(1ull << (w & 63));
      D.w_nbytes[w] -= res_nb(D, t);
      D.tdyn[t] |= TD_WHELD;
      if (D.holder_of[t] == w) {
        int h = -1;
        for (int b = 0; b < D.WB && h < 0; b++)
          if (row[b]) h = b * 64 + __builtin_ctzll(row[b]);
        D.holder_of[t] = h;
      }
    }
  }
  if (threadIdx.x == 0) {
    // the recommendations (:5235-5278): processing tasks, then the lost results; or a later
    // graph's runnable tasks
    long long sp = 0, nmark = 0;
    for (int i = 0; i < n_proc && D.ctl->error == 0; i++) {
      if (mode == LM_GRAPH) {
        loss_mark(D, nmark, proc[i], TD_READD);
        rec_push(D, sp, proc[i], RC_WAITING);
      } else if (mode == LM_RELEASE) {
        if (D.state[proc[i]] != S_PROCESSING) set_error(D, ERR_BAD_STATE, proc[i]);
        else rec_push(D, sp, proc[i], RC_RELEASED);
      } else if (killed && killed[i]) {
        loss_killed(D, O, sp, proc[i], w);  // KilledWorker: erred at once
      } else {
        rec_push(D, sp, proc[i], RC_RELEASED);
      }
    }
    for (int i = 0; i < n_held; i++) {
      const int t = held[i];
      bool any = false;
      for (int b = 0; b < D.WB && !any; b++) any = D.holders[(size_t)t * D.WB + b] != 0;
      if (!any) rec_push(D, sp, t, RC_RELEASED);
    }
    s_sp = sp;
    s_nmark = nmark;
  }
  __syncthreads();
  tree_rebuild_coop(D);
  int64_t stage_next = 0;  // lane 0's staging cursor
  while (true) {
    if (threadIdx.x == 0) {
      long long sp = s_sp, nmark = s_nmark;
      s_x = loss_machine(D, O, sp, nmark, w);
      s_sp = sp;
      s_nmark = nmark;
      c->pool_used = 0;
    }
    __syncthreads();
    const int x = s_x;
    if (x < 0) break;
    if (threadIdx.x < 64) candidate_row(D, x);  // decide_worker's candidates (who_has rows)
    __syncthreads();
    if (threadIdx.x == 0) {
      S.op = dispatch_prepare(D, x, S, &stage_next, dur);
      S.x = x;
    }
    __syncthreads();
    if (S.op != OP_NONE) dispatch_collective(D, S, &stage_next, dur);
    __syncthreads();
  }
  // the cascade's marks go; its placements become the placement log's tail (run_id order)
  __shared__ int64_t s_np;
  if (threadIdx.x == 0) s_np = stage_next;
  __syncthreads();
  const long long nmark = s_nmark;
  for (long long i = threadIdx.x; i < nmark; i += blockDim.x) {
    const int t = (int)D.release_key[i];
    D.tdyn[t] &= (uint8_t)~(TD_READD | TD_REWAIT);
  }
  for (int i = threadIdx.x; i < n_held; i += blockDim.x) D.tdyn[held[i]] &= (uint8_t)~TD_WHELD;
  const int64_t np = s_np;
  for (int64_t i = threadIdx.x; i < np; i += blockDim.x) {
    D.pl_task[pl0 + i] = D.st_task[i];
    D.pl_worker[pl0 + i] = D.st_worker[i];
    D.pl_comm[pl0 + i] = D.st_comm[i];
    D.pl_start[pl0 + i] = D.st_start[i];
    D.pl_wsnbytes[pl0 + i] = D.st_wsnbytes[i];
    D.pl_route[pl0 + i] = D.st_route[i];
  }
  if (threadIdx.x == 0) {
    c->n_placed = pl0 + np;
    *placed = np;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < (int)(sizeof(Ctl) / 4); i += blockDim.x) ((uint32_t*)ctl_g)[i] = ((const uint32_t*)&s_ctl)[i];
}

}  // namespace ev
}  // namespace dgp

namespace dgp {
namespace ev {

// ===================================================================== resync
// After a stimulus the engine does not model, the scheduler decided it itself; the host then
// hands over the scheduler's state (dgp_sync_*). Tasks: a sparse list of rows.
struct SyncTask {
  int32_t t, proc_on, remaining, waiters;
  int64_t nbytes;  // TaskState.nbytes (raw: -1 = never reported)
  int32_t hp, hn;  // who_has: holders [hp, hp + hn) of the holder list
  uint8_t state, lr, pad0, pad1;
  int32_t pad2;
};
static_assert(sizeof(SyncTask) == 40, "SyncTask layout is shared with the host");

__global__ void k_sync_tasks(const Dev* __restrict__ Dp, const SyncTask* __restrict__ rows, int n,
                             const int32_t* __restrict__ holders) {
  const Dev& D = *Dp;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const SyncTask r = rows[i];
    const int t = r.t;
    D.state[t] = r.state;
    D.remaining[t] = r.remaining;
    D.waiters[t] = r.waiters;
    D.proc_on[t] = r.proc_on;
    D.res_nbytes[t] = r.nbytes;
    D.cur_nbytes[t] = r.state == S_MEMORY ? nbv(D, r.nbytes) : -1;
    D.fr_mark[t] = -1;
    D.rel_mark[t] = -1;
    for (int b = 0; b < D.WB; b++) D.holders[(size_t)t * D.WB + b] = 0;
    int first = -1;
    for (int k = 0; k < r.hn; k++) {
      const int w = holders[r.hp + k];
      D.holders[(size_t)t * D.WB + (w >> 6)] |= 1ull << (w & 63);
      if (first < 0) first = w;
    }
    D.holder_of[t] = r.state == S_PROCESSING ? r.proc_on : first;
    D.tdyn[t] = (uint8_t)((r.lr ? TD_LR : 0) | (r.hn > 1 ? TD_MULTI : 0));
  }
}

// placements the scheduler made itself, appended to the placement log (their run identity)
__global__ void k_sync_placements(const Dev* __restrict__ Dp, const int32_t* __restrict__ task,
                                  const int32_t* __restrict__ worker, const int64_t* __restrict__ comm,
                                  const double* __restrict__ start, const int64_t* __restrict__ wsnb,
                                  const int8_t* __restrict__ route, int n) {
  const Dev& D = *Dp;
  const long long base = (long long)D.ctl->n_placed;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const long long pos = base + i;
    const int t = task[i];
    D.pl_task[pos] = t;
    D.pl_worker[pos] = worker[i];
    D.pl_comm[pos] = comm[i];
    D.pl_start[pos] = start[i];
    D.pl_wsnbytes[pos] = wsnb[i];
    D.pl_route[pos] = route[i];
  }
  __syncthreads();
  // run identity and holder: the last placement of each task wins (a suspended stimulus may
  // place one task twice), so one thread walks them in log order
  if (threadIdx.x == 0)
    for (int i = 0; i < n; i++) {
      D.run_id[task[i]] = (int32_t)(base + i);
      D.holder_of[task[i]] = worker[i];
    }
  if (threadIdx.x == 0) {
    D.ctl->n_placed = (unsigned long long)(base + n);
    D.pos->runid_upto = base + n;
  }
}

}  // namespace ev
}  // namespace dgp
