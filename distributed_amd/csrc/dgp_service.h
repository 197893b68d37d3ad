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

// One lane, in message order: every message is answered against the state left by all
// earlier messages (svc::answer, dgp_svcmsg.h). The stimuli accepted here only run after this
// kernel, so the first message whose answer could depend on them ends the call's batch; the
// host runs the accepted stimuli and calls again from there.
__global__ void k_svc_append(const Dev* __restrict__ Dp, const Msg* __restrict__ msgs, long long n,
                             int8_t* __restrict__ status, long long* __restrict__ consumed) {
  const Dev& D = *Dp;
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const long long len0 = *D.svc_len;
  long long len = len0;
  long long i = 0;
  for (; i < n; i++) {
    int8_t st = 0;
    if (!answer(D, msgs[i], len0, len, st)) break;  // answer after the accepted stimuli ran
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
