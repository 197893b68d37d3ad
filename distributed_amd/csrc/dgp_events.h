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
      for (long long i = 1; i < qn; i++) atomicAdd((unsigned long long*)&D.g_relwait[D.group[Q[i]]], (unsigned long long)-1ll);
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
