// dgplace service mode: the live scheduler's task-finished messages as stream stimuli.
// Included by dgplace.hip after dgp_stream.h.
//
// A replay (dgp_run_rounds) feeds the stream engine from its own placement log. In service
// mode the stimuli are the task-finished messages the caller hands over (dgp_tasks_finished),
// checked in arrival order exactly like Scheduler.handle_task_finished (scheduler.py:5783-5797)
// -> stimulus_task_finished (:5025-5092): stale, duplicate and already-in-memory reports are
// answered (free-keys / add-keys) instead of becoming completions. The accepted ones append to
// the stimulus log; the stream kernel then runs them (completion, frontier release, frontier
// placement, queue refill) with the engine state kept resident between calls.
#pragma once

namespace dgp {
namespace svc {

// answer to one task-finished message (the status codes of include/dgplace.h)
enum : int8_t {
  TF_ACCEPTED = 0,        // -> _transition(key, "memory", ...) (:5090): a completion stimulus
  TF_FREE_KEYS = 1,       // forgotten / released / queued / no-worker task, or a stale run
                          // from another worker (:5036-5049, :5065-5079): "free-keys" to the worker
  TF_ADD_KEYS = 2,        // the task is already in memory (:5082-5083): Scheduler.add_keys
  TF_RELEASE = 3,         // stale run_id from the worker the task is processing on (:5080-5081):
                          // the reference recommends "released" (re-placement); not run by the device
  TF_UNKNOWN_WORKER = 4,  // worker not in Scheduler.workers (:5786-5787): ignored
  TF_IMPOSSIBLE = 5,      // processing on another worker with the current run_id: the
                          // reference raises RuntimeError (:2398-2404)
  TF_UNSUPPORTED = 6,     // waiting -> memory with a matching run_id (_transition_waiting_memory)
};

// one message, packed by the host so the batch crosses PCIe in one copy
struct Msg {
  int32_t task, worker;
  int64_t run_id;
  int64_t nbytes;  // < 0: None (TaskState.set_nbytes is not called, :2424-2425)
  double start, stop;  // the "compute" startstop; NaN: none (no TaskPrefix EWMA step)
};
static_assert(sizeof(Msg) == 40, "Msg layout is shared with the host");

// One lane, in message order: every message is answered against the state left by all
// earlier messages. The stimuli accepted here only run after this kernel, so the first
// message whose answer could depend on them (a task that is waiting, queued or in memory,
// or that completed earlier in this batch: the frontier placement, the queue refill and
// the releases of those stimuli may change its state) ends the call's batch; the host runs
// the accepted stimuli and calls again from there. A processing task's run_id and worker
// change only through its own completion, and released / no-worker are final here.
__global__ void k_svc_append(const Dev* __restrict__ Dp, const Msg* __restrict__ msgs, long long n,
                             int8_t* __restrict__ status, long long* __restrict__ consumed) {
  const Dev& D = *Dp;
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const long long len0 = *D.svc_len;
  long long len = len0;
  long long i = 0;
  for (; i < n; i++) {
    const Msg m = msgs[i];
    int8_t st;
    if (m.worker < 0 || m.worker >= D.W) {
      st = TF_UNKNOWN_WORKER;
    } else if (m.task < 0 || m.task >= D.N) {
      st = TF_FREE_KEYS;  // ts is None
    } else {
      const int t = m.task;
      int s = D.state[t];
      const bool done_here = s == S_PROCESSING && D.sv_cseq[t] >= len0;  // completed in this call
      const bool stable = (s == S_PROCESSING && !done_here) || s == S_RELEASED || s == S_NO_WORKER;
      if (len > len0 && !stable) break;  // answer after the accepted stimuli ran
      if (s == S_RELEASED || s == S_QUEUED || s == S_NO_WORKER) {
        st = TF_FREE_KEYS;
      } else if ((int64_t)D.run_id[t] != m.run_id) {
        const bool on_w = s == S_PROCESSING && D.proc_on[t] == m.worker;
        st = on_w ? TF_RELEASE : TF_FREE_KEYS;
      } else if (s == S_MEMORY) {
        st = TF_ADD_KEYS;
      } else if (s == S_PROCESSING) {
        if (D.proc_on[t] != m.worker) {
          st = TF_IMPOSSIBLE;
        } else if (len >= D.sv_cap) {
          st = TF_IMPOSSIBLE;
          atomicCAS(&D.ctl->error, 0, (int)ERR_STAGE_CAP);
        } else {
          st = TF_ACCEPTED;
          D.sv_task[len] = t;
          D.sv_worker[len] = m.worker;
          D.sv_cseq[t] = (int32_t)len;
          D.holder_of[t] = m.worker;
          if (m.nbytes >= 0) D.res_nbytes[t] = m.nbytes;
          D.res_start[t] = m.start;
          D.res_stop[t] = m.stop;
          len++;
        }
      } else {
        st = TF_UNSUPPORTED;
      }
    }
    status[i] = st;
  }
  *D.svc_len = len;
  *consumed = i;
}

// run_id (placement-log position) and holder of the placements made since the last call:
// the update_graph stimulus and the round engine do not maintain them themselves
__global__ void k_set_runids(const Dev* __restrict__ Dp) {
  const Dev& D = *Dp;
  st::Pos* pos = D.pos;
  const long long a = pos->runid_upto, b = (long long)D.ctl->n_placed;
  for (long long i = a + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < b;
       i += (long long)gridDim.x * blockDim.x) {
    const int tk = D.pl_task[i];
    D.run_id[tk] = (int32_t)i;
    D.holder_of[tk] = D.pl_worker[i];
  }
}
__global__ void k_set_runids_done(const Dev* __restrict__ Dp) {
  if (threadIdx.x == 0) Dp->pos->runid_upto = (long long)Dp->ctl->n_placed;
}

// the round engine's completion batch = the stimuli appended since its last round
__global__ void k_svc_round_begin(const Dev* __restrict__ Dp, long long* consumed) {
  const Dev& D = *Dp;
  if (threadIdx.x != 0) return;
  Ctl* c = D.ctl;
  const long long a = *consumed, b = *D.svc_len;
  c->round_L = D.sv_task + a;
  c->round_n = b - a;
  *consumed = b;
  c->n_frontier = 0;
  c->pool_used = 0;
  c->round_counter++;
}

// one per-round snapshot of the service-mode state (the caller's round boundary)
__global__ void k_svc_snapshot_begin(const Dev* __restrict__ Dp) {
  if (threadIdx.x == 0) Dp->ctl->rounds_nonempty++;
}

}  // namespace svc
}  // namespace dgp
