// dgplace service messages: the task-finished message the host packs, the answer rules of
// Scheduler.stimulus_task_finished (scheduler.py:5025-5092) shared by the launch-per-call
// path (dgp_service.h k_svc_append) and the resident stream kernel (dgp_stream.h
// resident_serve), and the resident kernel's pinned mailbox. Included by dgp_stream.h.
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

// The answer to message m against the state the earlier messages left. len0: the stimulus
// log length when this batch (segment) began; len: its length now (an accepted message
// appends a stimulus). Returns false without answering when the answer depends on a stimulus
// accepted in this segment (its task is waiting, queued or in memory, or completed in this
// segment: those stimuli's frontier placement, refill and releases may change its state): the
// segment ends there and the message is answered after they ran. A processing task's run_id
// and worker change only through its own completion; released / no-worker are final here.
__device__ __forceinline__ bool answer(const Dev& D, const Msg& m, long long len0, long long& len, int8_t& st) {
  if (m.worker < 0 || m.worker >= D.W) {
    st = TF_UNKNOWN_WORKER;
    return true;
  }
  if (m.task < 0 || m.task >= D.N) {
    st = TF_FREE_KEYS;  // ts is None
    return true;
  }
  const int t = m.task;
  const int s = D.state[t];
  const bool done_here = s == S_PROCESSING && D.sv_cseq[t] >= len0;  // completed in this segment
  const bool stable = (s == S_PROCESSING && !done_here) || s == S_RELEASED || s == S_NO_WORKER;
  if (len > len0 && !stable) return false;
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
  return true;
}

// The resident service kernel's mailbox, in pinned, coherent host memory: the header, then
// cap messages, cap statuses and pl_cap (task, worker) pairs of the request's new placements;
// then, when the host asks for them (want_msgs), the compute-task message fields of those
// placements (_task_to_msg :3421-3450, as dgp_task_messages): per placement its first
// dependency entry (m_dptr, mp_cap + 1), per dependency entry the task, its first holder
// (m_hptr, md_cap + 1) and nbytes, and the holders (m_hidx, md_cap).
struct Mbox {
  unsigned long long req_seq;   // host: the request number, stored after the request
  unsigned long long done_seq;  // device: the last request answered (after its answers)
  long long n;                  // host: messages in the request
  long long cap, pl_cap;        // host: capacities of the arrays below
  long long n_placed;           // device: placement-log length after the request
  long long pl_from;            // device: log position of the first placement copied (-1: too many)
  int stop;                     // host: end the kernel
  int error;                    // device: the engine error that ended it (0: none)
  // device (100 MHz clock) per request: taken, stimuli appended (last segment), retired, published
  unsigned long long t_seen, t_app, t_ret, t_pub;
  // device: when each role last finished a batch (builder, prefetcher, registrar, executor
  // claim, executor done, sequencer retire, walker), copied at publish (diagnostics)
  unsigned long long t_role[7];
  long long mp_cap, md_cap;     // host: capacities of the message arrays (placements, entries)
  long long msg_from;           // device: log position of the first placement with message
                                // fields (-1: none this request: not asked for, or too many)
  int want_msgs;                // host: publish the message fields with the answers
};
__host__ __device__ inline size_t mbox_al(size_t b) { return (b + 15) & ~(size_t)15; }
__host__ __device__ inline size_t mbox_bytes(long long cap, long long pl_cap, long long mp_cap = 0,
                                             long long md_cap = 0) {
  return 256 + (size_t)cap * sizeof(Msg) + mbox_al((size_t)cap) + mbox_al((size_t)pl_cap * 8) +
         mbox_al((size_t)(mp_cap + 1) * 4) + mbox_al((size_t)md_cap * 4) + mbox_al((size_t)(md_cap + 1) * 4) +
         mbox_al((size_t)md_cap * 4) + (size_t)md_cap * 8;
}
__host__ __device__ inline Msg* mbox_msgs(Mbox* m) { return (Msg*)((char*)m + 256); }
__host__ __device__ inline int8_t* mbox_status(Mbox* m) { return (int8_t*)(mbox_msgs(m) + m->cap); }
__host__ __device__ inline int32_t* mbox_pl_task(Mbox* m) {
  return (int32_t*)((char*)mbox_status(m) + ((m->cap + 15) & ~15ll));
}
__host__ __device__ inline int32_t* mbox_pl_worker(Mbox* m) { return mbox_pl_task(m) + m->pl_cap; }
__host__ __device__ inline int32_t* mbox_m_dptr(Mbox* m) {
  return (int32_t*)((char*)mbox_pl_task(m) + mbox_al((size_t)m->pl_cap * 8));
}
__host__ __device__ inline int32_t* mbox_m_dtask(Mbox* m) {
  return (int32_t*)((char*)mbox_m_dptr(m) + mbox_al((size_t)(m->mp_cap + 1) * 4));
}
__host__ __device__ inline int32_t* mbox_m_hptr(Mbox* m) {
  return (int32_t*)((char*)mbox_m_dtask(m) + mbox_al((size_t)m->md_cap * 4));
}
__host__ __device__ inline int32_t* mbox_m_hidx(Mbox* m) {
  return (int32_t*)((char*)mbox_m_hptr(m) + mbox_al((size_t)(m->md_cap + 1) * 4));
}
__host__ __device__ inline int64_t* mbox_m_dnb(Mbox* m) {
  return (int64_t*)((char*)mbox_m_hidx(m) + mbox_al((size_t)m->md_cap * 4));
}
static_assert(sizeof(Mbox) <= 256, "mailbox header");

}  // namespace svc
}  // namespace dgp
