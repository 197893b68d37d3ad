// dgplace device side: state layout, the reference's placement semantics as device
// functions, and the kernels of one replay round. Included by dgplace.hip only.
//
// Reference: /root/reference/distributed/scheduler.py (SchedulerState) unless noted.
// Arithmetic follows CPython's evaluation order of the reference expressions; the
// translation unit is compiled with -ffp-contract=off (no fused multiply-add).
//
// Round structure (one wave of completions L[0..n)):
//   k_round_begin         reset per-round counters, n = |L|
//   k_frontier_release    all completions in parallel: publish the new replicas, atomic
//                         decrement of dependents' waiting_on and dependencies' waiters,
//                         tag every task with the position j of the completion that
//                         releases it (_add_to_memory :3298-3314)
//   k_candidate_commbytes one wave per newly ready task: candidate union + exact comm
//                         bytes per candidate (decide_worker :8571-8587, worker_objective
//                         :3136-3138) — HBM-bound gather of replica bitset rows
//   k_events              per completion stimulus j: the workers it may touch (its own,
//                         the holders of dependencies it releases, the candidates of the
//                         tasks it releases) and whether it needs global state
//   k_commit              ordered commit by deterministic reservation: in every step each
//                         pending stimulus reserves its workers with atomicMin(owner, j);
//                         a stimulus whose workers are all its own has no earlier pending
//                         stimulus touching them and commits concurrently with the others
//                         (identical to the sequential order). Stimuli that read global
//                         state (rootish / no-dependency placements, queue refill near
//                         exhaustion) run alone, cooperatively, in order.
// SchedulerState-global quantities that only feed check_idle_saturated's idle/saturated
// sets (total_occupancy :1877) are kept as an ordered record log and folded in by the
// log walker (k_walk) whenever a consumer needs them: before a global stimulus, for
// snapshots, and at the end of a replay.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dgp {

constexpr int PMAX = 8;        // distinct prefixes in one worker's task_prefix_count
constexpr int PMAX_G = 64;     // distinct prefixes in _task_prefix_count_global
constexpr int TOUCH_MAX = 24;  // workers one stimulus may reserve (more -> runs as global)
constexpr int CTA = 1024;      // threads of the commit / dispatch workgroup
constexpr int FL_MAX = 256;    // frontier tasks one global stimulus stages in LDS per chunk

enum : uint8_t { S_RELEASED = 0, S_WAITING, S_PROCESSING, S_QUEUED, S_NO_WORKER, S_MEMORY, S_ERRED };
enum : uint8_t { RF_RESTRICTED = 1, RF_LOOSE = 2 };
enum : uint8_t { TF_WANTED = 1, TF_ROOTISH = 2, TF_FORGOTTEN = 4 };  // TF_FORGOTTEN: left SchedulerState.tasks (resync)
// WF_PAUSED: the worker is not in SchedulerState.running (Status.paused, :5850-5883): never
// idle / saturated / in idle_task_count, never a decide_worker candidate
enum : uint8_t { WF_IDLE = 1, WF_SAT = 2, WF_ITC = 4, WF_PAUSED = 8 };
// per-task dynamic flags (Dev::tdyn): TD_LR the task is in its worker's long_running
// (add_to_long_running :747-757); TD_MULTI who_has is the task's holders bitset row (replicas
// beyond the one completion made, add_replica / remove_replica :3148-3159), not holder_of
// TD_READD / TD_REWAIT / TD_WHELD: marks of one worker-loss cascade (dgp_events.h), cleared by it
enum : uint8_t { TD_LR = 1, TD_MULTI = 2, TD_READD = 4, TD_REWAIT = 8, TD_WHELD = 16 };
// Dev::evf: which kinds of service events the engine has seen (each adds checks to the paths
// that must honour it; the replay workloads never set any)
enum : int32_t { EVF_MULTI = 1, EVF_LR = 2, EVF_PAUSED = 4 };
enum : uint8_t { EV_GLOBAL = 1 };
enum : int32_t { REC_NONE = 0, REC_COMPLETE = 1, REC_PLACE = 2 };
enum : int { ERR_NONE = 0, ERR_PREFIX_CAP, ERR_NO_CANDIDATES, ERR_BAD_STATE, ERR_QUEUE, ERR_POOL, ERR_GPREFIX_CAP,
             ERR_REC_CAP, ERR_STAGE_CAP, ERR_NO_WORKER, ERR_NEEDS_CAP,
             ERR_UNSUPPORTED = 20 };  // a service event the engine does not model (dgp_events.h);
                                      // 11..19 are the stream engine's SERR_* codes
enum : int { ROUTE_NONROOTISH = 0, ROUTE_ROOTISH_Q = 1, ROUTE_ROOTISH_NOQ = 2, ROUTE_FASTPATH = 3 };

// device-resident control block
struct Ctl {
  unsigned long long n_placed;    // placement log length (== next run_id)
  unsigned long long n_frontier;  // tasks released by the current round's completions
  unsigned long long pool_used;   // candidate pool entries used by the current round
  unsigned long long rec_used;    // record log length
  long long round_start, round_n; // current round = placement log slice
  long long round_counter;        // tags ready/release keys
  long long qhead, qlen;          // SchedulerState.queued (sorted array slice)
  long long n_tasks;              // SchedulerState.n_tasks
  long long n_itc;                // |idle_task_count| (eager)
  long long itc_slots;            // sum of _task_slots_available over idle_task_count (eager)
  long long n_unrunnable;
  // ---- walker state: SchedulerState as of record walk_pos
  unsigned long long walk_pos;
  long long n_idle, n_sat;        // |idle|, |saturated|
  double g_netocc;                // _network_occ_global
  int g_plen;                     // _task_prefix_count_global, insertion ordered
  int g_pfx[PMAX_G];
  long long g_pcnt[PMAX_G];
  // ----
  long long rounds_nonempty;      // rounds that completed at least one task
  const int32_t* round_L;         // completion list of the current round
  long long dr_steps;             // deterministic-reservation steps (diagnostics)
  unsigned long long prof2[16];   // exec_local_wave phase cycles (diagnostics)
  unsigned long long prof3[8];    // stream engine stall counters (diagnostics)
  unsigned long long prof[8];     // k_commit phase cycles (s_memtime): setup, local steps, global
                                  // stimuli, finish, walker, max step, -, -
  long long n_global_events;
  int error;
  int err_task;
};

// one sub-step of a stimulus that changes SchedulerState-global counts and is followed
// by check_idle_saturated(w) (completion: remove_from_processing; placement: add_to_processing)
struct Rec {
  int32_t kind;
  int32_t task;
  int32_t w;
  int32_t prefix;
  int64_t dnet;  // change of _network_occ_global
  double occ;    // WorkerState.occupancy of w at its check
  int32_t nproc; // len(w.processing) at its check
  int32_t pad;
};

namespace st {
struct SRec;
struct Pos;
}  // namespace st

struct Dev {
  int32_t N, W, WB, P, G, Wp;
  double bandwidth;  // SchedulerState.bandwidth: the config int, then the heartbeat EWMA (:4223-4226)
  int64_t default_data_size;
  double unknown_duration, saturation;
  int32_t sat_inf;
  int64_t total_nthreads;
  // graph (static)
  const int64_t* dep_ptr;
  const int32_t* dep_idx;
  const int64_t* dpt_ptr;
  const int32_t* dpt_idx;  // dependents, each row in ascending priority
  const int64_t* prio;
  const int32_t* prefix;
  const int32_t* group;
  const uint8_t* tflags;
  const int32_t* order;  // all tasks in ascending priority
  // synthetic completion reports
  int64_t* res_nbytes;
  double* res_start;
  double* res_stop;
  // task state
  uint8_t* state;
  int32_t* remaining;  // |waiting_on|
  int32_t* waiters;    // |waiters|
  int32_t* proc_on;    // processing_on, -1 when not processing
  int64_t* cur_nbytes;
  unsigned long long* holders;  // who_has bitsets [N][WB]
  unsigned long long* ready_key;
  unsigned long long* release_key;
  // candidate pool of newly ready tasks
  // worker restrictions (null: none): valid_workers(ts) resolved to worker indices
  // (scheduler.py:3043-3107), CSR ascending; restr_flags RF_RESTRICTED / RF_LOOSE
  const int64_t* restr_ptr;
  const int32_t* restr_idx;
  const uint8_t* restr_flags;
  // restrictions changed after the upload (dgp_update_restrictions: Scheduler.set_restrictions,
  // the shuffle's restrict_task): restr_ovr[t] >= 0 is task t's row in restr_pool (its length,
  // then its valid workers ascending) in place of the CSR row; null: none changed
  const int64_t* restr_ovr;
  const int32_t* restr_pool;
  int64_t* cand_off;
  int32_t* cand_n;
  int32_t* pool_w;
  int64_t* pool_comm;
  int64_t pool_cap;
  int32_t* frontier;
  // workers
  int32_t* w_nthreads;
  int32_t* w_cap;  // max(ceil(saturation * nthreads), 1)
  int32_t* w_nproc;
  int32_t* w_plen;
  int32_t* w_pfx;
  int32_t* w_pcnt;
  int64_t* w_netocc;
  int64_t* w_nbytes;
  uint8_t* w_flags;
  int64_t* w_itcslots;
  unsigned long long* w_lastcheck;  // record index of the worker's latest check
  uint32_t* w_needs;                // needs_what lines [W][NEEDS_W]
  double* t_key;                    // tournament tree over idle_task_count
  int32_t* t_idx;
  // prefixes
  double* pdur_cur;   // TaskPrefix.duration_average after all committed completions
  double* pdur_walk;  // ... as of the walker position
  double* pdur_pre;   // ... as of the stream prefetcher's position (it resolves each stimulus' durations)
  double* pmaxexec;   // TaskPrefix.max_exec_time (no heartbeats in the replay: -1)
  double* durv;       // per-round table: durations in effect at stimulus j, [n][P]
  // groups
  int64_t* g_size;
  int64_t* g_relwait;  // states["released"] + states["waiting"]
  int64_t* g_left;     // last_worker_tasks_left
  int32_t* g_lastw;    // last_worker
  // queue
  int32_t* qarr;
  // placement log
  int32_t* pl_task;
  int32_t* pl_worker;
  int64_t* pl_comm;
  double* pl_start;
  int64_t* pl_wsnbytes;
  int8_t* pl_route;
  int64_t pl_cap;  // placement-log capacity (>= N; grows in service sessions that re-place tasks)
  // record log
  Rec* rec;
  int64_t rec_cap;
  // per-round stimulus metadata
  int32_t* ev_w;
  int32_t* ev_nf;
  uint8_t* ev_flags;
  int32_t* ev_ntouch;
  int32_t* ev_touch;
  int64_t* ev_plbase;
  int64_t* ev_recbase;
  int32_t* ev_npl;
  int32_t* ev_pops;
  int32_t* ev_popmax;
  // per-round placement staging
  int32_t* st_task;
  int32_t* st_worker;
  int64_t* st_comm;
  double* st_start;
  int64_t* st_wsnbytes;
  int8_t* st_route;
  int64_t st_cap;
  // ready list of update_graph
  int32_t* ready;
  // snapshots
  int64_t snap_cap;
  int32_t* snap_nplaced;
  double* snap_occ;
  int64_t* snap_nbytes;
  int32_t* snap_nproc;
  uint8_t* snap_flags;
  int32_t* snap_nqueued;
  int32_t lds_workers;  // commit kernel: worker state lives in dynamic LDS
  int32_t needs_stream;  // needs_what lives in the stream engine's layout (gw_needs_saved / gw_needs_ext)
  Ctl* ctl;
  // ---- stream engine (dgp_stream.h)
  int32_t* gw_nproc;  // worker state in the stream layout when it does not fit in LDS
  uint16_t* gw_nthreads;
  uint16_t* gw_cap;
  uint32_t* gw_plen;
  uint32_t* gw_pcnt;
  int64_t* gw_netocc;
  int64_t* gw_nbytes;
  unsigned long long* gw_mask;  // in-flight stream slots touching each worker (bit per slot)
  uint32_t* gw_needs;
  uint8_t* gw_wflags;
  uint32_t* gw_needs_ext;    // needs_what overflow entries [W][NXW]
  unsigned long long* gw_held;  // [2][W] scratch of a global stimulus: held bytes, held deps per worker
  uint32_t* gw_needs_saved;  // needs_what lines between launches [W][NLW]
  int32_t* run_id;           // placement-log position of each placed task
  int32_t* holder_of;        // the worker a task runs / ran on (its single replica; one of them under TD_MULTI)
  uint8_t* tdyn;             // TD_LR / TD_MULTI per task
  int32_t evf;               // EVF_* seen so far
  int32_t* fr_mark;          // stimulus whose completion empties the task's waiting_on
  int32_t* rel_mark;         // stimulus whose completion empties the task's waiters
  uint4* desc;               // descriptor ring [DR][NE]
  double* dring;             // stimulus durations [DR][PX] when the graph has more prefixes than a descriptor carries
  int32_t* touch_ring;       // distinct workers each prefetched stimulus touches [DR][TMAX]
  uint2* thdr;               // per descriptor row: (flags, touched-worker count), written by PRE for REG
  int32_t* s2_task;  // per-slot staging of placements [WIN][PLC]
  int32_t* s2_worker;
  int64_t* s2_comm;
  double* s2_start;
  int64_t* s2_wsnb;
  int8_t* s2_route;
  st::SRec* srec;  // per-slot staging of records [WIN][PLC]
  st::SRec* rlog;  // the record log
  int64_t rlog_cap;
  st::Pos* pos;
  int32_t dbg_task;    // stream debug: dump the candidate keys of this frontier task
  double* dbgbuf;      // [64][8]
  int32_t pre_lead;  // stream: how far (stimuli) PRE may run ahead of SEQ (<= DR)
  int32_t dbg;  // stream debug: 1 every stimulus waits for all earlier ones, 2 every stimulus global
  // ---- the stimulus log the stream engine consumes. Replay mode: stimulus r completes
  // placement r (stim_task / stim_worker alias pl_task / pl_worker, cseq aliases run_id).
  // Service mode (dgp_tasks_finished): the accepted task-finished messages, in arrival order.
  const int32_t* stim_task;
  const int32_t* stim_worker;
  int32_t* cseq;         // stimulus index of each task's completion (-1: not completed)
  int32_t svc;           // 1: service mode (the launch ends at *svc_len)
  int32_t resident;      // service mode: the launch stays, answering requests from the mailbox
  void* mbox;            // resident service mailbox (dgp_service.h svc::Mbox, pinned host memory)
  long long* svc_len;    // service mode: stimulus-log length (device)
  int32_t* sv_task;      // service-mode stimulus log [sv_cap]
  int32_t* sv_worker;
  int32_t* sv_cseq;      // [N]
  int64_t sv_cap;
  // DGP_TRACE builds: per-stimulus lifecycle timestamps for stimuli [trace_lo, trace_lo + trace_n)
  unsigned long long* trace;
  long long trace_lo, trace_n;
};

// dynamic LDS of the commit kernel: owner[W] reservation table, then (lds_workers) the
// worker state arrays, each 16-byte aligned
extern __shared__ __attribute__((aligned(16))) char dgp_smem[];
__device__ __forceinline__ size_t lds_al(size_t b) { return (b + 15) & ~(size_t)15; }
// carve: owner[W] (16-byte aligned), then the worker arrays over Wa = W rounded up to 4
// workers, so every array starts 16-byte aligned. Byte offsets per worker:
constexpr int LDS_CUM[12] = {0, 4, 8, 12, 16, 16 + 4 * PMAX, 16 + 8 * PMAX, 24 + 8 * PMAX, 32 + 8 * PMAX,
                             40 + 8 * PMAX, 48 + 8 * PMAX, 49 + 8 * PMAX};
template <int K>
__device__ __forceinline__ char* lds_field_k(int W) {
  const size_t Wa = ((size_t)W + 3) & ~(size_t)3;
  return dgp_smem + lds_al((size_t)W * 4) + Wa * LDS_CUM[K];
}
__device__ __forceinline__ char* lds_field(int W, int k) {
  const size_t Wa = ((size_t)W + 3) & ~(size_t)3;
  return dgp_smem + lds_al((size_t)W * 4) + Wa * LDS_CUM[k];
}
#define WK_(D, f, k, T) ((D).lds_workers ? (T*)lds_field_k<k>((D).W) : (D).f)
#define WK_nthreads(D) WK_(D, w_nthreads, 0, int32_t)
#define WK_cap(D) WK_(D, w_cap, 1, int32_t)
#define WK_nproc(D) WK_(D, w_nproc, 2, int32_t)
#define WK_plen(D) WK_(D, w_plen, 3, int32_t)
#define WK_pfx(D) WK_(D, w_pfx, 4, int32_t)
#define WK_pcnt(D) WK_(D, w_pcnt, 5, int32_t)
#define WK_netocc(D) WK_(D, w_netocc, 6, int64_t)
#define WK_nbytes(D) WK_(D, w_nbytes, 7, int64_t)
#define WK_itcslots(D) WK_(D, w_itcslots, 8, int64_t)
#define WK_lastcheck(D) WK_(D, w_lastcheck, 9, unsigned long long)
#define WK_flags(D) WK_(D, w_flags, 10, uint8_t)

// ============================================================== small helpers

__device__ __forceinline__ int64_t get_nbytes(const Dev& D, int t) {  // TaskState.get_nbytes :1477
  int64_t v = D.cur_nbytes[t];
  return v >= 0 ? v : D.default_data_size;
}
__device__ __forceinline__ bool holds(const Dev& D, int d, int w) {
  return (D.holders[(size_t)d * D.WB + (w >> 6)] >> (w & 63)) & 1ull;
}
// w in d.who_has on the stream engine: holder_of, or the bitset row under TD_MULTI
__device__ __forceinline__ bool holds_any(const Dev& D, int d, int w) {
  if ((D.evf & EVF_MULTI) && (D.tdyn[d] & TD_MULTI)) return holds(D, d, w);
  return D.holder_of[d] == w;
}
// task x's valid workers (valid_workers :3043-3107 resolved on the host): idx[r0 .. r1)
struct RRow {
  const int32_t* idx;
  int64_t r0, r1;
};
__device__ __forceinline__ RRow restr_row(const Dev& D, int x) {
  if (D.restr_ovr) {
    const int64_t o = D.restr_ovr[x];
    if (o >= 0) return RRow{D.restr_pool, o + 1, o + 1 + D.restr_pool[o]};
  }
  return RRow{D.restr_idx, D.restr_ptr[x], D.restr_ptr[x + 1]};
}
// restricted and placed by decide_worker_non_rootish (a `_rootish` override wins, :2937)
__device__ __forceinline__ bool restricted_nonrootish(const Dev& D, int x) {
  return D.restr_flags && (D.restr_flags[x] & RF_RESTRICTED) && !(D.tflags[x] & TF_ROOTISH);
}
__device__ __forceinline__ void set_error(const Dev& D, int code, int task) {
  if (atomicCAS(&D.ctl->error, 0, code) == 0) D.ctl->err_task = task;
}
__device__ __forceinline__ double prefix_duration(const Dev& D, const double* dur, int p) {  // :1892-1899
  double d = dur[p];
  if (d < 0) {
    if (D.pmaxexec[p] > 0)
      d = 2 * D.pmaxexec[p];
    else
      d = D.unknown_duration;
  }
  return d;
}
// WorkerState.occupancy :840 -> _calc_occupancy :1884-1903 (dict insertion order)
__device__ double occupancy(const Dev& D, int w, const double* dur) {
  double res = 0.0;
  const int n = WK_plen(D)[w];
  const int* pf = WK_pfx(D) + (size_t)w * PMAX;
  const int* pc = WK_pcnt(D) + (size_t)w * PMAX;
  for (int i = 0; i < n; i++) res += prefix_duration(D, dur, pf[i]) * (double)pc[i];
  return res + (double)WK_netocc(D)[w] / (double)D.bandwidth;
}
// SchedulerState.total_occupancy :1877 at the walker position
__device__ double total_occupancy_walk(const Dev& D) {
  const Ctl* c = D.ctl;
  double res = 0.0;
  for (int i = 0; i < c->g_plen; i++) res += prefix_duration(D, D.pdur_walk, c->g_pfx[i]) * (double)c->g_pcnt[i];
  return res + c->g_netocc / (double)D.bandwidth;
}
__device__ __forceinline__ double ewma(double old, double duration) {  // TaskPrefix.add_duration :977-985
  return old < 0 ? duration : 0.5 * duration + 0.5 * old;
}

// insertion-ordered {prefix: count} dicts with delete-on-zero (:733-784)
__device__ bool wdict_inc(const Dev& D, int w, int p) {
  int* pf = WK_pfx(D) + (size_t)w * PMAX;
  int* pc = WK_pcnt(D) + (size_t)w * PMAX;
  int n = WK_plen(D)[w];
  for (int i = 0; i < n; i++)
    if (pf[i] == p) {
      pc[i]++;
      return true;
    }
  if (n == PMAX) return false;
  pf[n] = p;
  pc[n] = 1;
  WK_plen(D)[w] = n + 1;
  return true;
}
__device__ void wdict_dec(const Dev& D, int w, int p) {
  int* pf = WK_pfx(D) + (size_t)w * PMAX;
  int* pc = WK_pcnt(D) + (size_t)w * PMAX;
  int n = WK_plen(D)[w];
  for (int i = 0; i < n; i++)
    if (pf[i] == p) {
      if (--pc[i] == 0) {
        for (int k = i + 1; k < n; k++) {
          pf[k - 1] = pf[k];
          pc[k - 1] = pc[k];
        }
        WK_plen(D)[w] = n - 1;
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
  // cap[w] counts the worker's long-running tasks on top of max(ceil(sat * nthreads), 1)
  return (int64_t)WK_cap(D)[w] - (int64_t)WK_nproc(D)[w];
}
__device__ __forceinline__ bool worker_full(const Dev& D, int w) {  // :8770-8773
  if (D.sat_inf) return false;
  return task_slots_available(D, w) <= 0;
}

// ===================================================== idle_task_count (eager part)

// tournament tree: argmin over idle_task_count of (len(processing)/nthreads, index)
// (decide_worker_rootish_queuing_enabled :2230-2233). Only global stimuli use it; it is
// rebuilt cooperatively before they run and then maintained by their single lane.
__device__ void tree_update(const Dev& D, int w) {
  double key = (WK_flags(D)[w] & WF_ITC) ? (double)WK_nproc(D)[w] / (double)WK_nthreads(D)[w] : INFINITY;
  int pos = D.Wp + w;
  D.t_key[pos] = key;
  D.t_idx[pos] = w;
  double k = key;
  int i = w;
  // up the path 8 levels at a time: the 8 siblings are read first (the path's writes never
  // touch a sibling), one memory latency per 8 levels instead of one per level
  while (pos > 1) {
    double sk[8];
    int si[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {  // a level above the root reads node 3 (unused)
      const int p = max(pos >> j, 2);
      sk[j] = D.t_key[p ^ 1];
      si[j] = D.t_idx[p ^ 1];
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (pos > 1) {
        if (sk[j] < k || (sk[j] == k && si[j] < i)) {
          k = sk[j];
          i = si[j];
        }
        pos >>= 1;
        D.t_key[pos] = k;
        D.t_idx[pos] = i;
      }
    }
  }
}
__device__ __attribute__((noinline)) void tree_rebuild_coop(const Dev& D) {  // all threads of the block
  for (int i = threadIdx.x; i < D.Wp; i += blockDim.x) {
    int pos = D.Wp + i;
    bool on = i < D.W && (WK_flags(D)[i] & WF_ITC);
    D.t_key[pos] = on ? (double)WK_nproc(D)[i] / (double)WK_nthreads(D)[i] : INFINITY;
    D.t_idx[pos] = i;
  }
  __threadfence_block();
  __syncthreads();
  for (int half = D.Wp >> 1; half >= 1; half >>= 1) {
    for (int pos = half + threadIdx.x; pos < 2 * half; pos += blockDim.x) {
      double a = D.t_key[2 * pos], b = D.t_key[2 * pos + 1];
      int ia = D.t_idx[2 * pos], ib = D.t_idx[2 * pos + 1];
      bool right = b < a || (b == a && ib < ia);
      D.t_key[pos] = right ? b : a;
      D.t_idx[pos] = right ? ib : ia;
    }
    __threadfence_block();
    __syncthreads();
  }
}

// the idle_task_count part of check_idle_saturated (:2992-2995): depends only on w
__device__ void itc_check(const Dev& D, int w, bool maintain_tree) {
  uint8_t fl = WK_flags(D)[w];
  bool on = !worker_full(D, w) && !(fl & WF_PAUSED);  // ... and ws.status == running (:2992)
  bool was = (fl & WF_ITC) != 0;
  if (on != was) {
    WK_flags(D)[w] = on ? (fl | WF_ITC) : (fl & ~WF_ITC);
    atomicAdd((unsigned long long*)&D.ctl->n_itc, on ? 1ull : (unsigned long long)-1ll);
  }
  int64_t contrib = on ? task_slots_available(D, w) : 0;
  int64_t delta = contrib - WK_itcslots(D)[w];
  if (delta) atomicAdd((unsigned long long*)&D.ctl->itc_slots, (unsigned long long)delta);
  WK_itcslots(D)[w] = contrib;
  if (maintain_tree) tree_update(D, w);
}

// ====================================================== record log and its walker

// write the record of one sub-step and note it as w's latest check_idle_saturated
__device__ void emit(const Dev& D, int64_t slot, int32_t kind, int32_t task, int32_t w, int32_t prefix, int64_t dnet,
                     const double* dur) {
  if (slot >= D.rec_cap) {
    set_error(D, ERR_REC_CAP, task);
    return;
  }
  Rec r;
  r.kind = kind;
  r.task = task;
  r.w = w;
  r.prefix = prefix;
  r.dnet = dnet;
  r.occ = occupancy(D, w, dur);
  r.nproc = WK_nproc(D)[w];
  r.pad = 0;
  D.rec[slot] = r;
  WK_lastcheck(D)[w] = (unsigned long long)slot;
}

// the idle / saturated part of check_idle_saturated (:2949-2991 + is_unoccupied :2997)
__device__ void walk_flags(const Dev& D, int w, double occ, int64_t p) {
  Ctl* c = D.ctl;
  int64_t nt = WK_nthreads(D)[w];
  uint8_t fl = WK_flags(D)[w];
  bool idle = false, sat = false;
  double avg = -1;
  if (fl & WF_PAUSED) {
    // not running: idle.pop, saturated.discard (:2975-2977)
  } else if (p < nt) {
    idle = true;
  } else {
    avg = total_occupancy_walk(D) / (double)D.total_nthreads;
    idle = occ < (double)nt * avg / 2;
  }
  if (!idle && p > nt && !(fl & WF_PAUSED)) {
    double pending = occ * (double)(p - nt) / (double)(p * nt);
    if (0.4 < pending) {
      if (avg < 0) avg = total_occupancy_walk(D) / (double)D.total_nthreads;
      sat = pending > 1.9 * avg;
    }
  }
  if (idle != ((fl & WF_IDLE) != 0)) c->n_idle += idle ? 1 : -1;
  if (sat != ((fl & WF_SAT) != 0)) c->n_sat += sat ? 1 : -1;
  WK_flags(D)[w] = (fl & ~(WF_IDLE | WF_SAT)) | (idle ? WF_IDLE : 0) | (sat ? WF_SAT : 0);
}

// fold records [walk_pos, end) into the walker state (single lane)
__device__ __attribute__((noinline)) void walk_to(const Dev& D, unsigned long long end) {
  Ctl* c = D.ctl;
  for (unsigned long long i = c->walk_pos; i < end; i++) {
    Rec r = D.rec[i];
    if (r.kind == REC_NONE) continue;
    if (r.kind == REC_COMPLETE) {
      D.pdur_walk[r.prefix] = ewma(D.pdur_walk[r.prefix], D.res_stop[r.task] - D.res_start[r.task]);
      gdict_dec(D, r.prefix);
    } else {
      if (!gdict_inc(D, r.prefix)) set_error(D, ERR_GPREFIX_CAP, r.task);
    }
    c->g_netocc += (double)r.dnet;
    if (WK_lastcheck(D)[r.w] == i) walk_flags(D, r.w, r.occ, r.nproc);
  }
  if (end > c->walk_pos) c->walk_pos = end;
}

// ============================================================ objective & needs

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
__device__ __forceinline__ Obj objective(const Dev& D, int w, int64_t comm, const double* dur) {
  double stack_time = occupancy(D, w, dur) / (double)WK_nthreads(D)[w];
  double start_time = stack_time + (double)comm / (double)D.bandwidth;
  return Obj{start_time, WK_nbytes(D)[w], w};
}
__device__ int64_t comm_bytes(const Dev& D, int t, int w) {  // worker_objective's sum :3136-3138
  int64_t comm = 0;
  for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
    int d = D.dep_idx[k];
    if (!holds(D, d, w)) comm += get_nbytes(D, d);
  }
  return comm;
}
// needs_what[w][d] > 0 <=> another dependent of d is processing on w (w does not hold d)
__device__ bool needed_elsewhere(const Dev& D, int d, int w, int except) {
  for (int64_t k = D.dpt_ptr[d]; k < D.dpt_ptr[d + 1]; k++) {
    int x = D.dpt_idx[k];
    if (x != except && D.proc_on[x] == w) return true;
  }
  return false;
}

// WorkerState.needs_what (:800-823) as one 128-byte line per worker: up to NEEDS_W - 1
// entries (d << 8 | count), 0 = empty. Only the stimulus owning the worker touches it.
// A worker that needs more dependencies at once (a shuffle barrier, rootish pile-ups)
// switches to exact scans of the dependents' processing_on (needed_elsewhere) until
// it has nothing processing again.
constexpr int NEEDS_W = 32;
constexpr uint32_t NEEDS_OVF = 0xffffffffu;  // in the last slot: scan mode
__device__ __forceinline__ uint32_t* needs_line(const Dev& D, int w) { return D.w_needs + (size_t)w * NEEDS_W; }
__device__ __forceinline__ bool needs_overflowed(const Dev& D, int w) {
  return needs_line(D, w)[NEEDS_W - 1] == NEEDS_OVF;
}
// The same operations on the stream engine's layout (dgp_stream.h needs_inc / needs_dec /
// needs_reset, one lane instead of a wave): gw_needs_saved[w] = SNLW - 1 entries
// (d << 8 | count) and a control word (entry count << 8, or SNL_OVF: scan mode), the rest in
// gw_needs_ext[w] (SNXW entries). The update_graph dispatcher and the service-event
// cascades place with these when the stream engine owns the worker state.
constexpr int SNLW = 12, SNXW = 52;
constexpr uint32_t SNL_OVF = 0xffffffffu;
__device__ __forceinline__ int64_t res_nb(const Dev& D, int d) {
  const int64_t v = D.res_nbytes[d];
  return v >= 0 ? v : D.default_data_size;
}
__device__ int64_t sneeds_inc(const Dev& D, int w, int d, int t) {
  uint32_t* L = D.gw_needs_saved + (size_t)w * SNLW;
  uint32_t* X = D.gw_needs_ext + (size_t)w * SNXW;
  const int64_t nb = res_nb(D, d);
  const uint32_t ctl = L[SNLW - 1];
  if (ctl == SNL_OVF) return needed_elsewhere(D, d, w, t) ? 0 : nb;
  int used = 0, empty = -1;
  for (int i = 0; i < SNLW - 1; i++) {
    const uint32_t e = L[i];
    if (e != 0 && (e >> 8) == (uint32_t)d) {
      if ((e & 0xffu) == 0xffu) {
        set_error(D, ERR_BAD_STATE, d);
        return 0;
      }
      L[i] = e + 1;
      return 0;
    }
    if (e != 0) used++;
    else if (empty < 0) empty = i;
  }
  const int ext = (int)(ctl >> 8) - used;
  int xempty = 0;
  if (ext > 0) {
    xempty = -1;
    for (int i = 0; i < SNXW; i++) {
      const uint32_t e = X[i];
      if (e != 0 && (e >> 8) == (uint32_t)d) {
        if ((e & 0xffu) == 0xffu) {
          set_error(D, ERR_BAD_STATE, d);
          return 0;
        }
        X[i] = e + 1;
        return 0;
      }
      if (e == 0 && xempty < 0) xempty = i;
    }
  }
  if (empty >= 0) {
    L[empty] = ((uint32_t)d << 8) | 1u;
    L[SNLW - 1] = ctl + 0x100u;
    return nb;
  }
  if (ext < SNXW) {
    X[xempty] = ((uint32_t)d << 8) | 1u;
    L[SNLW - 1] = ctl + 0x100u;
    return nb;
  }
  L[SNLW - 1] = SNL_OVF;  // full: scan mode
  return nb;
}
__device__ int64_t sneeds_dec(const Dev& D, int w, int d, int t) {
  uint32_t* L = D.gw_needs_saved + (size_t)w * SNLW;
  uint32_t* X = D.gw_needs_ext + (size_t)w * SNXW;
  const int64_t nb = res_nb(D, d);
  const uint32_t ctl = L[SNLW - 1];
  if (ctl == SNL_OVF) return needed_elsewhere(D, d, w, t) ? 0 : nb;
  int used = 0;
  for (int i = 0; i < SNLW - 1; i++) {
    const uint32_t e = L[i];
    if (e != 0 && (e >> 8) == (uint32_t)d) {
      const uint32_t v = e - 1;
      const bool gone = (v & 0xffu) == 0;
      L[i] = gone ? 0u : v;
      if (gone) L[SNLW - 1] = ctl - 0x100u;
      return gone ? nb : 0;
    }
    used += e != 0;
  }
  if ((int)(ctl >> 8) - used > 0)
    for (int i = 0; i < SNXW; i++) {
      const uint32_t e = X[i];
      if (e != 0 && (e >> 8) == (uint32_t)d) {
        const uint32_t v = e - 1;
        const bool gone = (v & 0xffu) == 0;
        X[i] = gone ? 0u : v;
        if (gone) L[SNLW - 1] = ctl - 0x100u;
        return gone ? nb : 0;
      }
    }
  if (D.evf & EVF_MULTI) return 0;  // a replica event may have removed the entry (add_replica :831-834)
  set_error(D, ERR_BAD_STATE, d);
  return 0;
}
__device__ void sneeds_reset(const Dev& D, int w) {  // a worker with nothing processing needs nothing
  uint32_t* L = D.gw_needs_saved + (size_t)w * SNLW;
  const uint32_t ctl = L[SNLW - 1];
  if (ctl == SNL_OVF || (ctl >> 8) != 0)
    for (int i = 0; i < SNXW; i++) D.gw_needs_ext[(size_t)w * SNXW + i] = 0u;
  for (int i = 0; i < SNLW; i++) L[i] = 0u;
}

// _inc_needs_replica: bytes w newly needs (0 if d was needed already); t = task being placed
__device__ int64_t needs_inc(const Dev& D, int w, int d, int t) {
  if (D.needs_stream) return sneeds_inc(D, w, d, t);
  uint32_t* line = needs_line(D, w);
  if (line[NEEDS_W - 1] != NEEDS_OVF) {
    const uint32_t key = (uint32_t)d << 8;
    int empty = -1;
    for (int q = 0; q < NEEDS_W / 4; q++) {
      uint4 v = reinterpret_cast<const uint4*>(line)[q];
      uint32_t e[4] = {v.x, v.y, v.z, v.w};
      for (int i = 0; i < 4; i++) {
        int slot = 4 * q + i;
        if (e[i] != 0 && (e[i] & ~0xffu) == key && slot < NEEDS_W - 1) {
          if ((e[i] & 0xffu) != 0xffu) {
            line[slot] = e[i] + 1;
            return 0;
          }
          line[NEEDS_W - 1] = NEEDS_OVF;  // count saturated: scan mode
          return needed_elsewhere(D, d, w, t) ? 0 : get_nbytes(D, d);
        }
        if (e[i] == 0 && empty < 0 && slot < NEEDS_W - 1) empty = slot;
      }
    }
    if (empty >= 0) {
      line[empty] = key | 1u;
      return get_nbytes(D, d);
    }
    line[NEEDS_W - 1] = NEEDS_OVF;  // full: scan mode
  }
  return needed_elsewhere(D, d, w, t) ? 0 : get_nbytes(D, d);
}
// _dec_needs_replica (only when d is in needs_what); t = task leaving w (processing_on cleared)
__device__ int64_t needs_dec(const Dev& D, int w, int d, int t) {
  if (D.needs_stream) return sneeds_dec(D, w, d, t);
  uint32_t* line = needs_line(D, w);
  if (line[NEEDS_W - 1] != NEEDS_OVF) {
    const uint32_t key = (uint32_t)d << 8;
    for (int q = 0; q < NEEDS_W / 4; q++) {
      uint4 v = reinterpret_cast<const uint4*>(line)[q];
      uint32_t e[4] = {v.x, v.y, v.z, v.w};
      for (int i = 0; i < 4; i++)
        if (e[i] != 0 && (e[i] & ~0xffu) == key) {
          uint32_t ne = e[i] - 1;
          bool gone = (ne & 0xffu) == 0;
          line[4 * q + i] = gone ? 0u : ne;
          return gone ? get_nbytes(D, d) : 0;
        }
    }
    return 0;
  }
  return (!holds(D, d, w) && !needed_elsewhere(D, d, w, t)) ? get_nbytes(D, d) : 0;
}
// a worker with nothing processing needs nothing: leave scan mode
__device__ __forceinline__ void needs_maybe_reset(const Dev& D, int w) {
  if (D.needs_stream) {
    if (WK_nproc(D)[w] == 0) sneeds_reset(D, w);
    return;
  }
  uint32_t* line = needs_line(D, w);
  if (line[NEEDS_W - 1] == NEEDS_OVF && WK_nproc(D)[w] == 0)
    for (int i = 0; i < NEEDS_W; i++) line[i] = 0;
}

// ================================================================= mutations

// processing->memory of t on w (:2366-2442) up to the frontier; returns the record slot used
__device__ void do_completion(const Dev& D, int t, int w, int64_t rslot, const double* dur) {
  int p = D.prefix[t];
  D.proc_on[t] = -1;  // _exit_processing_common -> remove_from_processing :759-771
  wdict_dec(D, w, p);
  WK_nproc(D)[w]--;
  int64_t dnet = 0;
  if (D.dep_ptr[t + 1] > D.dep_ptr[t]) {
    for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) dnet -= needs_dec(D, w, D.dep_idx[k], t);
    WK_netocc(D)[w] += dnet;
  }
  needs_maybe_reset(D, w);
  emit(D, rslot, REC_COMPLETE, t, w, p, dnet, dur);  // check_idle_saturated(ws) :3276
  // add_replica (:3148): the who_has bit and nbytes were published by k_frontier_release
  WK_nbytes(D)[w] += get_nbytes(D, t);
  D.state[t] = S_MEMORY;
}

// _transition_memory_released (:2444-2505) -> remove_all_replicas (:3161-3171)
__device__ void release_task(const Dev& D, int t) {
  int64_t nb = get_nbytes(D, t);
  unsigned long long* row = D.holders + (size_t)t * D.WB;
  for (int wd = 0; wd < D.WB; wd++) {
    unsigned long long bits = row[wd];
    while (bits) {
      int b = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      WK_nbytes(D)[wd * 64 + b] -= nb;
    }
    row[wd] = 0;
  }
  D.state[t] = S_RELEASED;
  atomicAdd((unsigned long long*)&D.g_relwait[D.group[t]], 1ull);
}

// the releases of completion stimulus (t, key): popped before the frontier (LIFO)
__device__ void do_releases(const Dev& D, int t, unsigned long long key) {
  for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
    int d = D.dep_idx[k];
    if (D.release_key[d] == key && D.waiters[d] == 0 && !(D.tflags[d] & TF_WANTED) && D.state[d] == S_MEMORY)
      release_task(D, d);
  }
  if (D.dpt_ptr[t + 1] == D.dpt_ptr[t] && !(D.tflags[t] & TF_WANTED)) release_task(D, t);
}

__device__ __forceinline__ bool is_frontier(const Dev& D, int x, unsigned long long key) {
  return D.ready_key[x] == key && D.state[x] == S_WAITING && D.remaining[x] == 0;
}

// _add_to_processing :3199-3256 (+ WorkerState.add_to_processing :733): record, mutate
__device__ void do_place(const Dev& D, int t, int w, int route, int64_t comm, int64_t plslot, int64_t rslot,
                         const double* dur, bool maintain_tree) {
  if (comm < 0) comm = comm_bytes(D, t, w);
  Obj o = objective(D, w, comm, dur);
  D.st_task[plslot] = t;
  D.st_worker[plslot] = w;
  D.st_comm[plslot] = comm;
  D.st_start[plslot] = o.start;
  D.st_wsnbytes[plslot] = WK_nbytes(D)[w];
  D.st_route[plslot] = (int8_t)route;
  int p = D.prefix[t];
  if (!wdict_inc(D, w, p)) set_error(D, ERR_PREFIX_CAP, t);
  WK_nproc(D)[w]++;
  int64_t dnet = 0;
  if (D.dep_ptr[t + 1] > D.dep_ptr[t]) {
    for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
      int d = D.dep_idx[k];
      if (!holds(D, d, w)) dnet += needs_inc(D, w, d, t);
    }
    WK_netocc(D)[w] += dnet;
  }
  if (t >= 0) {
    D.proc_on[t] = w;
    if (D.state[t] == S_WAITING) atomicAdd((unsigned long long*)&D.g_relwait[D.group[t]], (unsigned long long)-1ll);
    D.state[t] = S_PROCESSING;
  }
  emit(D, rslot, REC_PLACE, t, w, p, dnet, dur);  // check_idle_saturated(ws) :3212
  itc_check(D, w, maintain_tree);
  atomicAdd((unsigned long long*)&D.ctl->n_tasks, 1ull);
}

// ======================================================= local stimulus (one lane)

// a completion stimulus whose placements only read the workers it reserved
__device__ void exec_local(const Dev& D, int j, int t, int w, unsigned long long key, const double* dur,
                           int64_t plbase, int64_t recbase, int popmax, int pop_prefix) {
  do_completion(D, t, w, recbase, dur);
  itc_check(D, w, false);
  do_releases(D, t, key);
  int64_t npl = 0, nrec = 1;
  for (int64_t k = D.dpt_ptr[t]; k < D.dpt_ptr[t + 1]; k++) {
    int x = D.dpt_idx[k];
    if (!is_frontier(D, x, key)) continue;
    // decide_worker (:8550-8593) over the precomputed candidates
    int n = D.cand_n[x];
    int64_t off = D.cand_off[x];
    if (n <= 0) {
      set_error(D, ERR_NO_CANDIDATES, x);
      return;
    }
    int best = D.pool_w[off];
    int64_t bcomm = D.pool_comm[off];
    if (n > 1) {
      Obj bo = objective(D, best, bcomm, dur);
      for (int i = 1; i < n; i++) {
        Obj o = objective(D, D.pool_w[off + i], D.pool_comm[off + i], dur);
        if (obj_less(o, bo)) {
          bo = o;
          best = o.w;
          bcomm = D.pool_comm[off + i];
        }
      }
    }
    do_place(D, x, best, ROUTE_NONROOTISH, bcomm, plbase + npl, recbase + nrec, dur, false);
    npl++;
    nrec++;
  }
  // stimulus_queue_slots_maybe_opened (:4983): with a non-empty queue every other
  // worker is full, so the open slots are w's; the queued tasks are resolved in order later
  int pops = 0;
  if (popmax > 0 && (WK_flags(D)[w] & WF_ITC)) {
    int64_t slots = task_slots_available(D, w);
    for (int64_t i = 0; i < slots && pops < popmax; i++) {
      // place a placeholder (task -1) of the queue's prefix on w: route rootish-queuing
      int64_t plslot = plbase + npl, rslot = recbase + nrec;
      Obj o = objective(D, w, 0, dur);
      D.st_task[plslot] = -1;
      D.st_worker[plslot] = w;
      D.st_comm[plslot] = 0;
      D.st_start[plslot] = o.start;
      D.st_wsnbytes[plslot] = WK_nbytes(D)[w];
      D.st_route[plslot] = ROUTE_ROOTISH_Q;
      if (!wdict_inc(D, w, pop_prefix)) set_error(D, ERR_PREFIX_CAP, -1);
      WK_nproc(D)[w]++;
      emit(D, rslot, REC_PLACE, -1, w, pop_prefix, 0, dur);
      itc_check(D, w, false);
      atomicAdd((unsigned long long*)&D.ctl->n_tasks, 1ull);
      npl++;
      nrec++;
      pops++;
    }
  }
  D.ev_npl[j] = (int32_t)npl;
  D.ev_pops[j] = pops;
}


// ================================================= local stimulus, one wave per stimulus
//
// Memory discipline (gfx950 counts loads and stores on one in-order vmcnt): every global
// load of the stimulus is issued before any global store, the loads are spread over the
// wave's lanes, worker state is touched only through typed LDS (ds_*) or global
// accessors, and all global stores happen in one final phase.

template <bool LW>
struct WS;  // worker-state accessors: LW = state in the commit kernel's LDS carve
template <>
struct WS<true> {
  static __device__ __forceinline__ int32_t* nthreads(const Dev& D) { return (int32_t*)lds_field_k<0>(D.W); }
  static __device__ __forceinline__ int32_t* cap(const Dev& D) { return (int32_t*)lds_field_k<1>(D.W); }
  static __device__ __forceinline__ int32_t* nproc(const Dev& D) { return (int32_t*)lds_field_k<2>(D.W); }
  static __device__ __forceinline__ int32_t* plen(const Dev& D) { return (int32_t*)lds_field_k<3>(D.W); }
  static __device__ __forceinline__ int32_t* pfx(const Dev& D) { return (int32_t*)lds_field_k<4>(D.W); }
  static __device__ __forceinline__ int32_t* pcnt(const Dev& D) { return (int32_t*)lds_field_k<5>(D.W); }
  static __device__ __forceinline__ int64_t* netocc(const Dev& D) { return (int64_t*)lds_field_k<6>(D.W); }
  static __device__ __forceinline__ int64_t* nbytes(const Dev& D) { return (int64_t*)lds_field_k<7>(D.W); }
  static __device__ __forceinline__ int64_t* itcslots(const Dev& D) { return (int64_t*)lds_field_k<8>(D.W); }
  static __device__ __forceinline__ unsigned long long* lastcheck(const Dev& D) {
    return (unsigned long long*)lds_field_k<9>(D.W);
  }
  static __device__ __forceinline__ uint8_t* flags(const Dev& D) { return (uint8_t*)lds_field_k<10>(D.W); }
};
template <>
struct WS<false> {
  static __device__ __forceinline__ int32_t* nthreads(const Dev& D) { return D.w_nthreads; }
  static __device__ __forceinline__ int32_t* cap(const Dev& D) { return D.w_cap; }
  static __device__ __forceinline__ int32_t* nproc(const Dev& D) { return D.w_nproc; }
  static __device__ __forceinline__ int32_t* plen(const Dev& D) { return D.w_plen; }
  static __device__ __forceinline__ int32_t* pfx(const Dev& D) { return D.w_pfx; }
  static __device__ __forceinline__ int32_t* pcnt(const Dev& D) { return D.w_pcnt; }
  static __device__ __forceinline__ int64_t* netocc(const Dev& D) { return D.w_netocc; }
  static __device__ __forceinline__ int64_t* nbytes(const Dev& D) { return D.w_nbytes; }
  static __device__ __forceinline__ int64_t* itcslots(const Dev& D) { return D.w_itcslots; }
  static __device__ __forceinline__ unsigned long long* lastcheck(const Dev& D) { return D.w_lastcheck; }
  static __device__ __forceinline__ uint8_t* flags(const Dev& D) { return D.w_flags; }
};

template <bool LW>
__device__ __forceinline__ double occ_w(const Dev& D, int w, const double* dur) {  // _calc_occupancy :1884
  using S = WS<LW>;
  double res = 0.0;
  const int n = S::plen(D)[w];
  const int32_t* pf = S::pfx(D) + (size_t)w * PMAX;
  const int32_t* pc = S::pcnt(D) + (size_t)w * PMAX;
  for (int i = 0; i < n; i++) res += prefix_duration(D, dur, pf[i]) * (double)pc[i];
  return res + (double)S::netocc(D)[w] / (double)D.bandwidth;
}
template <bool LW>
__device__ __forceinline__ bool wd_inc(const Dev& D, int w, int p) {
  using S = WS<LW>;
  int32_t* pf = S::pfx(D) + (size_t)w * PMAX;
  int32_t* pc = S::pcnt(D) + (size_t)w * PMAX;
  int n = S::plen(D)[w];
  for (int i = 0; i < n; i++)
    if (pf[i] == p) {
      pc[i]++;
      return true;
    }
  if (n == PMAX) return false;
  pf[n] = p;
  pc[n] = 1;
  S::plen(D)[w] = n + 1;
  return true;
}
template <bool LW>
__device__ __forceinline__ void wd_dec(const Dev& D, int w, int p) {
  using S = WS<LW>;
  int32_t* pf = S::pfx(D) + (size_t)w * PMAX;
  int32_t* pc = S::pcnt(D) + (size_t)w * PMAX;
  int n = S::plen(D)[w];
  for (int i = 0; i < n; i++)
    if (pf[i] == p) {
      if (--pc[i] == 0) {
        for (int k2 = i + 1; k2 < n; k2++) {
          pf[k2 - 1] = pf[k2];
          pc[k2 - 1] = pc[k2];
        }
        S::plen(D)[w] = n - 1;
      }
      return;
    }
}
// idle_task_count part of check_idle_saturated; the global counters change by the returned deltas
template <bool LW>
__device__ __forceinline__ void itc_local(const Dev& D, int w, int64_t& d_itc, int64_t& d_slots) {
  using S = WS<LW>;
  int64_t slots = D.sat_inf ? 0 : (int64_t)S::cap(D)[w] - (int64_t)S::nproc(D)[w];
  bool on = D.sat_inf || slots > 0;
  uint8_t fl = S::flags(D)[w];
  bool was = (fl & WF_ITC) != 0;
  if (on != was) {
    S::flags(D)[w] = on ? (fl | WF_ITC) : (fl & ~WF_ITC);
    d_itc += on ? 1 : -1;
  }
  int64_t contrib = on ? slots : 0;
  d_slots += contrib - S::itcslots(D)[w];
  S::itcslots(D)[w] = contrib;
}

__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// one needs_what line cached in the lanes (entry `lane`), see NeedsLine layout above
struct LaneLine {
  int w;        // worker, -1 unused
  uint32_t e;   // this lane's entry
  bool dirty;
};

template <bool LW>
__device__ void exec_local_wave(const Dev& D, int j, int t, int w, unsigned long long key, const double* dur,
                                int64_t plbase, int64_t recbase, int popmax, int pop_prefix) {
  using S = WS<LW>;
  const int lane = threadIdx.x & 63;
  unsigned long long _ts = __builtin_amdgcn_s_memtime();
  // ------------------------------------------------------------ gather (loads only)
  const int64_t d0 = D.dep_ptr[t], d1 = D.dep_ptr[t + 1];
  const int64_t e0 = D.dpt_ptr[t], e1 = D.dpt_ptr[t + 1];
  const int k = (int)(d1 - d0), f = (int)(e1 - e0);
  const int p = D.prefix[t];
  const int64_t nbt = get_nbytes(D, t);
  const bool t_wanted = (D.tflags[t] & TF_WANTED) != 0;
  const int dl = lane < k ? D.dep_idx[d0 + lane] : -1;
  const int xl = lane < f ? D.dpt_idx[e0 + lane] : -1;
  LaneLine ln[9];
  ln[0].w = w;
  ln[0].e = lane < NEEDS_W ? needs_line(D, w)[lane] : 0u;
  ln[0].dirty = false;
  for (int q = 1; q < 9; q++) {
    ln[q].w = -1;
    ln[q].e = 0;
    ln[q].dirty = false;
  }
  const int64_t nbd = dl >= 0 ? get_nbytes(D, dl) : 0;
  const bool hd = dl >= 0 ? holds(D, dl, w) : true;
  const bool reld = dl >= 0 && D.release_key[dl] == key && D.waiters[dl] == 0 && !(D.tflags[dl] & TF_WANTED);
  const bool fr = xl >= 0 && is_frontier(D, xl, key);
  const unsigned long long frmask = __ballot(fr);
  const unsigned long long relmask = __ballot(reld);
  const bool self_rel = f == 0 && !t_wanted;
  const bool w_ovf = __shfl(ln[0].e, NEEDS_W - 1) == NEEDS_OVF;
  { unsigned long long _t = __builtin_amdgcn_s_memtime(); if (lane == 0) atomicAdd(&D.ctl->prof2[0], _t - _ts); _ts = _t; }
  // records (lane r holds record r) and placements (lane q holds placement q)
  int r_kind = REC_NONE, r_task = -1, r_w = 0, r_prefix = 0, r_np = 0;
  int64_t r_dnet = 0;
  double r_occ = 0;
  int q_task = -1, q_w = 0;
  int64_t q_comm = 0, q_wsnb = 0;
  double q_start = 0;
  int8_t q_route = 0;
  int nrec = 0, npl = 0;
  int64_t d_itc = 0, d_slots = 0;
  int xw = -1;  // in a frontier task's lane: the worker it was placed on

  // ------------------------------------------------------ completion (:2366-2442)
  int64_t dnet = 0;
  if (k > 0) {
    if (!w_ovf) {
      for (int i = 0; i < k; i++) {  // _dec_needs_replica for every dependency in needs_what
        const uint32_t key_i = (uint32_t)__shfl(dl, i) << 8;
        const unsigned long long m = __ballot(lane < NEEDS_W - 1 && ln[0].e != 0 && (ln[0].e & ~0xffu) == key_i);
        if (m) {
          const int ml = __ffsll((long long)m) - 1;
          if (lane == ml) {
            ln[0].e -= 1;
            if ((ln[0].e & 0xffu) == 0) ln[0].e = 0;
          }
          ln[0].dirty = true;
          if (__shfl(ln[0].e, ml) == 0) dnet -= __shfl(nbd, i);
        }
      }
    } else {
      const int64_t mine = (dl >= 0 && !hd && !needed_elsewhere(D, dl, w, t)) ? nbd : 0;
      dnet = -wave_sum64(mine);
    }
  }
  if (lane == 0) {
    wd_dec<LW>(D, w, p);
    S::nproc(D)[w]--;
    S::netocc(D)[w] += dnet;
  }
  __builtin_amdgcn_wave_barrier();
  if (w_ovf && S::nproc(D)[w] == 0) {  // nothing processing: leave scan mode
    ln[0].e = 0;
    ln[0].dirty = true;
  }
  {
    const double o = occ_w<LW>(D, w, dur);
    const int np = S::nproc(D)[w];
    if (lane == 0) {
      r_kind = REC_COMPLETE;
      r_task = t;
      r_w = w;
      r_prefix = p;
      r_dnet = dnet;
      r_occ = o;
      r_np = np;
      S::lastcheck(D)[w] = (unsigned long long)recbase;
      itc_local<LW>(D, w, d_itc, d_slots);
      S::nbytes(D)[w] += nbt;  // add_replica
    }
    nrec = 1;
  }
  __builtin_amdgcn_wave_barrier();
  { unsigned long long _t = __builtin_amdgcn_s_memtime(); if (lane == 0) atomicAdd(&D.ctl->prof2[1], _t - _ts); _ts = _t; }
  // releases (popped before the frontier); remove_all_replicas -> holders' nbytes
  {
    unsigned long long rm = relmask;
    while (rm) {
      const int i = __ffsll((long long)rm) - 1;
      rm &= rm - 1;
      const int d = __shfl(dl, i);
      const int64_t nb = __shfl(nbd, i);
      for (int wd = lane; wd < D.WB; wd += 64) {
        unsigned long long bits = D.holders[(size_t)d * D.WB + wd];
        while (bits) {
          const int b = __ffsll((long long)bits) - 1;
          bits &= bits - 1;
          atomicAdd((unsigned long long*)&S::nbytes(D)[wd * 64 + b], (unsigned long long)(-nb));
        }
      }
    }
    if (self_rel && lane == 0) S::nbytes(D)[w] -= nbt;  // t's only replica is on w
  }
  __builtin_amdgcn_wave_barrier();

  { unsigned long long _t = __builtin_amdgcn_s_memtime(); if (lane == 0) atomicAdd(&D.ctl->prof2[2], _t - _ts); _ts = _t; }
  // ------------------------------------------ frontier placements, ascending priority
  unsigned long long fm = frmask;
  while (fm) {
    const int fi = __ffsll((long long)fm) - 1;
    fm &= fm - 1;
    const int x = __shfl(xl, fi);
    const int px = D.prefix[x];
    const int cn = D.cand_n[x];
    const int64_t co = D.cand_off[x];
    const int64_t xd0 = D.dep_ptr[x], xd1 = D.dep_ptr[x + 1];
    const int kx = (int)(xd1 - xd0);
    const int cl = lane < cn ? D.pool_w[co + lane] : -1;
    const int64_t cm = lane < cn ? D.pool_comm[co + lane] : 0;
    const int dxl = lane < kx ? D.dep_idx[xd0 + lane] : -1;
    const int64_t nbx = dxl >= 0 ? get_nbytes(D, dxl) : 0;
  { unsigned long long _t = __builtin_amdgcn_s_memtime(); if (lane == 0) atomicAdd(&D.ctl->prof2[3], _t - _ts); _ts = _t; }
    // decide_worker (:8550-8593): argmin of worker_objective over the candidates
    Obj o{INFINITY, INT64_MAX, INT32_MAX};
    if (cl >= 0) o = Obj{occ_w<LW>(D, cl, dur) / (double)S::nthreads(D)[cl] + (double)cm / (double)D.bandwidth,
                         S::nbytes(D)[cl], cl};
    int64_t ocm = cm;
    for (int off = 32; off > 0; off >>= 1) {
      Obj q{__shfl_xor(o.start, off), __shfl_xor(o.nbytes, off), __shfl_xor(o.w, off)};
      const int64_t qc = __shfl_xor(ocm, off);
      if (obj_less(q, o)) {
        o = q;
        ocm = qc;
      }
    }
    const int c = o.w;
  { unsigned long long _t = __builtin_amdgcn_s_memtime(); if (lane == 0) atomicAdd(&D.ctl->prof2[4], _t - _ts); _ts = _t; }
    const bool hx = dxl >= 0 ? holds(D, dxl, c) : true;
    // the needs_what line of c in the lanes
    int li = -1;
    for (int q = 0; q < 9; q++)
      if (li < 0 && ln[q].w == c) li = q;
    if (li < 0)
      for (int q = 1; q < 9; q++)
        if (li < 0 && ln[q].w < 0) {
          li = q;
          ln[q].w = c;
          ln[q].e = lane < NEEDS_W ? needs_line(D, c)[lane] : 0u;
          ln[q].dirty = false;
        }
    // (k_events caps the frontier at 8 tasks, so a slot is always free)
    uint32_t e = 0;
    for (int q = 0; q < 9; q++)
      if (q == li) e = ln[q].e;
    bool ovf = __shfl(e, NEEDS_W - 1) == NEEDS_OVF;
  { unsigned long long _t = __builtin_amdgcn_s_memtime(); if (lane == 0) atomicAdd(&D.ctl->prof2[5], _t - _ts); _ts = _t; }
    int64_t dnx = 0;
    bool dirty = false;
    for (int i = 0; i < kx && !ovf; i++) {  // _inc_needs_replica
      if (__shfl(hx, i)) continue;
      const uint32_t key_i = (uint32_t)__shfl(dxl, i) << 8;
      const unsigned long long m = __ballot(lane < NEEDS_W - 1 && e != 0 && (e & ~0xffu) == key_i);
      if (m) {
        const int ml = __ffsll((long long)m) - 1;
        if ((__shfl(e, ml) & 0xffu) == 0xffu) {
          ovf = true;
          break;
        }
        if (lane == ml) e += 1;
      } else {
        const unsigned long long em = __ballot(lane < NEEDS_W - 1 && e == 0);
        if (!em) {
          ovf = true;
          break;
        }
        if (lane == __ffsll((long long)em) - 1) e = key_i | 1u;
        dnx += __shfl(nbx, i);
      }
      dirty = true;
    }
    if (ovf) {
      // scan mode for c: publish the processing_on of this stimulus' earlier placements
      // first (the scan reads them), then decide each dependency exactly
      if (lane == NEEDS_W - 1) e = NEEDS_OVF;
      dirty = true;
      if (xw >= 0) D.proc_on[xl] = xw;
      __threadfence_block();
      const int64_t mine = (dxl >= 0 && !hx && !needed_elsewhere(D, dxl, c, x)) ? nbx : 0;
      dnx = wave_sum64(mine);
    }
    for (int q = 0; q < 9; q++)
      if (q == li) {
        ln[q].e = e;
        ln[q].dirty = ln[q].dirty || dirty;
      }
    // _add_to_processing (:3199): record, WorkerState.add_to_processing, check_idle_saturated
    if (lane == npl) {
      q_task = x;
      q_w = c;
      q_comm = ocm;
      q_start = o.start;
      q_wsnb = o.nbytes;
      q_route = ROUTE_NONROOTISH;
    }
    if (lane == 0) {
      if (!wd_inc<LW>(D, c, px)) set_error(D, ERR_PREFIX_CAP, x);
      S::nproc(D)[c]++;
      S::netocc(D)[c] += dnx;
    }
    __builtin_amdgcn_wave_barrier();
    {
      const double oc = occ_w<LW>(D, c, dur);
      const int np = S::nproc(D)[c];
      if (lane == nrec) {
        r_kind = REC_PLACE;
        r_task = x;
        r_w = c;
        r_prefix = px;
        r_dnet = dnx;
        r_occ = oc;
        r_np = np;
      }
      if (lane == 0) {
        S::lastcheck(D)[c] = (unsigned long long)(recbase + nrec);
        itc_local<LW>(D, c, d_itc, d_slots);
      }
    }
    if (lane == fi) xw = c;
    npl++;
    nrec++;
    __builtin_amdgcn_wave_barrier();
  { unsigned long long _t = __builtin_amdgcn_s_memtime(); if (lane == 0) atomicAdd(&D.ctl->prof2[6], _t - _ts); _ts = _t; }
  }
  // ----------------- queue refill: with a non-empty queue only w can have open slots
  int pops = 0;
  if (popmax > 0) {
    int64_t slots = S::cap(D)[w] - (int64_t)S::nproc(D)[w];
    if (!(S::flags(D)[w] & WF_ITC)) slots = 0;
    for (int64_t i = 0; i < slots && pops < popmax; i++) {
      const double o0 = occ_w<LW>(D, w, dur);
      const int64_t nb0 = S::nbytes(D)[w];
      if (lane == npl) {
        q_task = -1;  // resolved in queue order after the commit
        q_w = w;
        q_comm = 0;
        q_start = o0 / (double)S::nthreads(D)[w];
        q_wsnb = nb0;
        q_route = ROUTE_ROOTISH_Q;
      }
      if (lane == 0) {
        if (!wd_inc<LW>(D, w, pop_prefix)) set_error(D, ERR_PREFIX_CAP, -1);
        S::nproc(D)[w]++;
      }
      __builtin_amdgcn_wave_barrier();
      const double o1 = occ_w<LW>(D, w, dur);
      const int np = S::nproc(D)[w];
      if (lane == nrec) {
        r_kind = REC_PLACE;
        r_task = -1;
        r_w = w;
        r_prefix = pop_prefix;
        r_dnet = 0;
        r_occ = o1;
        r_np = np;
      }
      if (lane == 0) {
        S::lastcheck(D)[w] = (unsigned long long)(recbase + nrec);
        itc_local<LW>(D, w, d_itc, d_slots);
      }
      __builtin_amdgcn_wave_barrier();
      npl++;
      nrec++;
      pops++;
    }
  }

  { unsigned long long _t = __builtin_amdgcn_s_memtime(); if (lane == 0) atomicAdd(&D.ctl->prof2[7], _t - _ts); _ts = _t; }
  // ----------------------------------------------------------------- store phase
  if (lane == 0) {
    D.state[t] = self_rel ? S_RELEASED : S_MEMORY;
    D.proc_on[t] = -1;
    if (self_rel) atomicAdd((unsigned long long*)&D.g_relwait[D.group[t]], 1ull);
    D.ev_npl[j] = npl;
    D.ev_pops[j] = pops;
    if (d_itc) atomicAdd((unsigned long long*)&D.ctl->n_itc, (unsigned long long)d_itc);
    if (d_slots) atomicAdd((unsigned long long*)&D.ctl->itc_slots, (unsigned long long)d_slots);
    atomicAdd((unsigned long long*)&D.ctl->n_tasks, (unsigned long long)npl);
  }
  if (self_rel)
    for (int wd = lane; wd < D.WB; wd += 64) D.holders[(size_t)t * D.WB + wd] = 0;
  if (reld) {
    D.state[dl] = S_RELEASED;
    for (int wd = 0; wd < D.WB; wd++) D.holders[(size_t)dl * D.WB + wd] = 0;
    atomicAdd((unsigned long long*)&D.g_relwait[D.group[dl]], 1ull);
  }
  if (xw >= 0) {
    D.state[xl] = S_PROCESSING;
    D.proc_on[xl] = xw;
    atomicAdd((unsigned long long*)&D.g_relwait[D.group[xl]], (unsigned long long)-1ll);
  }
  for (int q = 0; q < 9; q++)
    if (ln[q].w >= 0 && __ballot(ln[q].dirty) && lane < NEEDS_W) needs_line(D, ln[q].w)[lane] = ln[q].e;
  if (lane < nrec) {
    Rec r;
    r.kind = r_kind;
    r.task = r_task;
    r.w = r_w;
    r.prefix = r_prefix;
    r.dnet = r_dnet;
    r.occ = r_occ;
    r.nproc = r_np;
    r.pad = 0;
    D.rec[recbase + lane] = r;
  }
  if (lane < npl) {
    const int64_t sl = plbase + lane;
    D.st_task[sl] = q_task;
    D.st_worker[sl] = q_w;
    D.st_comm[sl] = q_comm;
    D.st_start[sl] = q_start;
    D.st_wsnbytes[sl] = q_wsnb;
    D.st_route[sl] = q_route;
  }
  { unsigned long long _t = __builtin_amdgcn_s_memtime(); if (lane == 0) atomicAdd(&D.ctl->prof2[8], _t - _ts); _ts = _t; }
}

// ======================================================= block-level collectives

// exclusive prefix sum of one int64 per thread over the block; *total = block sum
__device__ int64_t block_excl_scan(int64_t v, int64_t* total) {
  __shared__ int64_t s_w[CTA / 64];
  __shared__ int64_t s_tot;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int64_t incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    int64_t u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int i = 0; i < nw; i++) {
      int64_t t = s_w[i];
      s_w[i] = run;
      run += t;
    }
    s_tot = run;
  }
  __syncthreads();
  int64_t res = s_w[wid] + incl - v;
  *total = s_tot;
  __syncthreads();
  return res;
}

struct ArgBest {
  Obj o;
  int64_t comm;
};
// block argmin of worker_objective; threads with w < 0 contribute nothing
__device__ ArgBest block_argmin(Obj o, int64_t comm, bool valid) {
  __shared__ double s_start[CTA / 64];
  __shared__ int64_t s_nb[CTA / 64];
  __shared__ int32_t s_w[CTA / 64];
  __shared__ int64_t s_comm[CTA / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (!valid) {
    o.start = INFINITY;
    o.nbytes = INT64_MAX;
    o.w = INT32_MAX;
  }
  for (int off = 32; off > 0; off >>= 1) {
    Obj q{__shfl_xor(o.start, off), __shfl_xor(o.nbytes, off), __shfl_xor(o.w, off)};
    int64_t qc = __shfl_xor(comm, off);
    if (obj_less(q, o)) {
      o = q;
      comm = qc;
    }
  }
  if (lane == 0) {
    s_start[wid] = o.start;
    s_nb[wid] = o.nbytes;
    s_w[wid] = o.w;
    s_comm[wid] = comm;
  }
  __syncthreads();
  ArgBest b{Obj{s_start[0], s_nb[0], s_w[0]}, s_comm[0]};
  for (int i = 1; i < nw; i++) {
    Obj q{s_start[i], s_nb[i], s_w[i]};
    if (obj_less(q, b.o)) {
      b.o = q;
      b.comm = s_comm[i];
    }
  }
  __syncthreads();
  return b;
}

// ordered list of the workers in the pool `idle if idle else all` into LDS (first `cap`)
__device__ int64_t gather_pool(const Dev& D, bool use_idle, int32_t* list, int cap) {
  int64_t base = 0;
  for (int w0 = 0; w0 < D.W; w0 += blockDim.x) {
    int w = w0 + threadIdx.x;
    bool in = w < D.W && (use_idle ? (WK_flags(D)[w] & WF_IDLE) : !(WK_flags(D)[w] & WF_PAUSED));
    int64_t tot;
    int64_t pos = block_excl_scan(in ? 1 : 0, &tot);
    if (in && base + pos < cap) list[base + pos] = w;
    base += tot;
  }
  __syncthreads();
  return base;
}

// ====================================================== global stimulus (cooperative)

// state shared by the lanes of a cooperative global stimulus / the update_graph dispatcher
struct CoopShared {
  int op;
  int x;
  int best;
  int64_t best_comm;
  int nlist;
  int pos;
  int done;
  int32_t list[FL_MAX];
  int32_t pool[32];
  int64_t pool_n;
};
enum : int { OP_NONE = 0, OP_ARGMIN_POOL, OP_FASTPATH, OP_KTH, OP_RESTRICTED, OP_RUNNING };

// eager application of a sub-step (global stimuli): what the walker would do with its record
__device__ void apply_now(const Dev& D, int32_t kind, int t, int w, int p, int64_t dnet, const double* dur) {
  Ctl* c = D.ctl;
  if (kind == REC_COMPLETE) {
    D.pdur_walk[p] = ewma(D.pdur_walk[p], D.res_stop[t] - D.res_start[t]);
    gdict_dec(D, p);
  } else if (!gdict_inc(D, p)) {
    set_error(D, ERR_GPREFIX_CAP, t);
  }
  c->g_netocc += (double)dnet;
  walk_flags(D, w, occupancy(D, w, dur), WK_nproc(D)[w]);
}

// _add_to_processing for global stimuli: staging slot from the overflow area
__device__ void place_eager(const Dev& D, int t, int w, int route, int64_t comm, int64_t* stage_next,
                            const double* dur) {
  int64_t slot = (*stage_next)++;
  if (slot >= D.st_cap) {
    set_error(D, ERR_STAGE_CAP, t);
    return;
  }
  // do_place emits into the record log; global stimuli apply instead (records slot unused)
  if (comm < 0) comm = comm_bytes(D, t, w);
  Obj o = objective(D, w, comm, dur);
  D.st_task[slot] = t;
  D.st_worker[slot] = w;
  D.st_comm[slot] = comm;
  D.st_start[slot] = o.start;
  D.st_wsnbytes[slot] = WK_nbytes(D)[w];
  D.st_route[slot] = (int8_t)route;
  int p = D.prefix[t];
  if (!wdict_inc(D, w, p)) set_error(D, ERR_PREFIX_CAP, t);
  WK_nproc(D)[w]++;
  int64_t dnet = 0;
  if (D.dep_ptr[t + 1] > D.dep_ptr[t]) {
    for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
      int d = D.dep_idx[k];
      if (!holds(D, d, w)) dnet += needs_inc(D, w, d, t);
    }
    WK_netocc(D)[w] += dnet;
  }
  D.proc_on[t] = w;
  if (D.state[t] == S_WAITING) atomicAdd((unsigned long long*)&D.g_relwait[D.group[t]], (unsigned long long)-1ll);
  D.state[t] = S_PROCESSING;
  apply_now(D, REC_PLACE, t, w, p, dnet, dur);
  itc_check(D, w, true);
  D.ctl->n_tasks++;
}

__device__ void queue_insert(const Dev& D, int t) {  // HeapSet.add as a sorted array
  Ctl* c = D.ctl;
  long long lo = c->qhead, pos = c->qhead + c->qlen;
  int64_t pr = D.prio[t];
  while (pos > lo && D.prio[D.qarr[pos - 1]] > pr) {
    D.qarr[pos] = D.qarr[pos - 1];
    pos--;
  }
  D.qarr[pos] = t;
  c->qlen++;
}

// lane 0: first half of _transition_waiting_processing (:2313-2336) for task x. Either
// finishes it (returns OP_NONE) or names the collective it needs.
__device__ int dispatch_prepare(const Dev& D, int x, CoopShared& S, int64_t* stage_next, const double* dur) {
  Ctl* c = D.ctl;
  if (D.tflags[x] & TF_ROOTISH) {
    if (D.sat_inf) {  // decide_worker_rootish_queuing_disabled :2135-2193
      int gi = D.group[x];
      // last_worker, while it has tasks left and still runs (:2168-2171)
      if (D.g_lastw[gi] >= 0 && D.g_left[gi] != 0 && !(WK_flags(D)[D.g_lastw[gi]] & WF_PAUSED)) {
        int w = D.g_lastw[gi];
        D.g_lastw[gi] = D.g_relwait[gi] > 1 ? w : -1;
        D.g_left[gi] -= 1;
        place_eager(D, x, w, ROUTE_ROOTISH_NOQ, -1, stage_next, dur);
        return OP_NONE;
      }
      return OP_ARGMIN_POOL;
    }
    // decide_worker_rootish_queuing_enabled :2195-2245
    if (c->n_itc == 0) {  // -> queued (:2761)
      D.state[x] = S_QUEUED;
      atomicAdd((unsigned long long*)&D.g_relwait[D.group[x]], (unsigned long long)-1ll);
      queue_insert(D, x);
      return OP_NONE;
    }
    place_eager(D, x, D.t_idx[1], ROUTE_ROOTISH_Q, -1, stage_next, dur);
    return OP_NONE;
  }
  if (restricted_nonrootish(D, x)) return OP_RESTRICTED;  // decide_worker with valid_workers
  if (D.dep_ptr[x + 1] > D.dep_ptr[x]) {  // decide_worker over the candidates
    int n = D.cand_n[x];
    int64_t off = D.cand_off[x];
    if (n <= 0) {
      // every holder paused: valid_workers = running (:2262-2266), candidates & valid empty ->
      // candidates = valid (:8575-8582)
      if (D.evf & EVF_PAUSED) return OP_RUNNING;
      set_error(D, ERR_NO_CANDIDATES, x);
      return OP_NONE;
    }
    int best = D.pool_w[off];
    int64_t bcomm = D.pool_comm[off];
    if (n > 1) {
      Obj bo = objective(D, best, bcomm, dur);
      for (int i = 1; i < n; i++) {
        Obj o = objective(D, D.pool_w[off + i], D.pool_comm[off + i], dur);
        if (obj_less(o, bo)) {
          bo = o;
          best = o.w;
          bcomm = D.pool_comm[off + i];
        }
      }
    }
    place_eager(D, x, best, ROUTE_NONROOTISH, bcomm, stage_next, dur);
    return OP_NONE;
  }
  // no-dependency fast path :2283-2305 (pool = idle, else running)
  bool use_idle = c->n_idle > 0;
  if (!use_idle && (D.evf & EVF_PAUSED)) return OP_KTH;  // a paused / removed worker: the pool is counted there
  int64_t n = use_idle ? c->n_idle : D.W;
  if (n >= 20 && !use_idle) {
    place_eager(D, x, (int)(c->n_tasks % n), ROUTE_FASTPATH, -1, stage_next, dur);
    return OP_NONE;
  }
  return n < 20 ? OP_FASTPATH : OP_KTH;
}

// all lanes: the collective part, then lane 0 finishes the placement
__device__ __attribute__((noinline)) void dispatch_collective(const Dev& D, CoopShared& S, int64_t* stage_next, const double* dur) {
  int op = S.op, x = S.x;
  Ctl* c = D.ctl;
  if (op == OP_RUNNING) {  // decide_worker's argmin over every running worker
    Obj best{INFINITY, INT64_MAX, INT32_MAX};
    int64_t bcomm = 0;
    bool have = false;
    for (int w = threadIdx.x; w < D.W; w += blockDim.x) {
      if (WK_flags(D)[w] & WF_PAUSED) continue;
      const int64_t cm = comm_bytes(D, x, w);
      const Obj o = objective(D, w, cm, dur);
      if (!have || obj_less(o, best)) {
        best = o;
        bcomm = cm;
        have = true;
      }
    }
    ArgBest b = block_argmin(best, bcomm, have);
    if (threadIdx.x == 0) {
      if (b.o.w == INT32_MAX) {  // no running worker: no-worker
        D.state[x] = S_NO_WORKER;
        atomicAdd((unsigned long long*)&D.g_relwait[D.group[x]], (unsigned long long)-1ll);
        c->n_unrunnable++;
      } else {
        place_eager(D, x, b.o.w, ROUTE_NONROOTISH, b.comm, stage_next, dur);
      }
    }
  } else if (op == OP_ARGMIN_POOL) {
    bool use_idle = c->n_idle > 0;
    Obj best{INFINITY, INT64_MAX, INT32_MAX};
    int64_t bcomm = 0;
    bool have = false;
    for (int w = threadIdx.x; w < D.W; w += blockDim.x) {
      if (use_idle ? !(WK_flags(D)[w] & WF_IDLE) : (WK_flags(D)[w] & WF_PAUSED)) continue;  // idle, else running
      int64_t cm = comm_bytes(D, x, w);
      Obj o = objective(D, w, cm, dur);
      if (!have || obj_less(o, best)) {
        best = o;
        bcomm = cm;
        have = true;
      }
    }
    ArgBest b = block_argmin(best, bcomm, have);
    if (threadIdx.x == 0) {
      int gi = D.group[x];
      int w = b.o.w;
      if (w == INT32_MAX) {
        D.state[x] = S_NO_WORKER;
        atomicAdd((unsigned long long*)&D.g_relwait[gi], (unsigned long long)-1ll);
        c->n_unrunnable++;
      } else {
        D.g_left[gi] = (int64_t)floor(((double)D.g_size[gi] / (double)D.total_nthreads) * (double)WK_nthreads(D)[w]);
        D.g_lastw[gi] = D.g_relwait[gi] > 1 ? w : -1;
        D.g_left[gi] -= 1;
        place_eager(D, x, w, ROUTE_ROOTISH_NOQ, b.comm, stage_next, dur);
      }
    }
  } else if (op == OP_RESTRICTED) {
    // decide_worker (:8550-8593) with valid = valid_workers(ts) (:3043-3107; every worker
    // runs here): candidates = who_has of the dependencies & valid; if none, valid; if
    // that is empty too, the loose retry without restrictions (:8584-8586) or None ->
    // no-worker (:2761-2782). The argmin of worker_objective decides (a single candidate
    // is its own argmin).
    const RRow rr = restr_row(D, x);
    const int64_t r0 = rr.r0, r1 = rr.r1;
    const int64_t d0 = D.dep_ptr[x], d1 = D.dep_ptr[x + 1];
    auto held = [&](int w) {
      for (int64_t k = d0; k < d1; k++)
        if (holds(D, D.dep_idx[k], w)) return true;
      return false;
    };
    // valid_workers & running: a paused / removed worker is never valid (:3099-3105)
    auto run = [&](int w) { return !(WK_flags(D)[w] & WF_PAUSED); };
    int64_t nval = 0;
    for (int64_t i0 = r0; i0 < r1; i0 += blockDim.x) {
      const int64_t i = i0 + threadIdx.x;
      int64_t t1;
      block_excl_scan(i < r1 && run(rr.idx[i]) ? 1 : 0, &t1);
      nval += t1;
    }
    int64_t tot = 0;
    for (int64_t i0 = r0; i0 < r1; i0 += blockDim.x) {
      const int64_t i = i0 + threadIdx.x;
      int64_t t1;
      block_excl_scan(i < r1 && run(rr.idx[i]) && held(rr.idx[i]) ? 1 : 0, &t1);
      tot += t1;
    }
    // 0: valid & holders, 1: valid, 2: holders (loose), 3: every worker (loose), 4: none
    int mode = tot > 0 ? 0 : (nval > 0 ? 1 : 4);
    if (mode == 4 && (D.restr_flags[x] & RF_LOOSE)) {
      int64_t nh = 0;
      for (int w0 = 0; w0 < D.W; w0 += blockDim.x) {
        const int w = w0 + threadIdx.x;
        int64_t t1;
        block_excl_scan(w < D.W && run(w) && held(w) ? 1 : 0, &t1);
        nh += t1;
      }
      mode = nh > 0 ? 2 : 3;
    }
    Obj best{INFINITY, INT64_MAX, INT32_MAX};
    int64_t bcomm = 0;
    bool have = false;
    auto consider = [&](int w) {
      const int64_t cm = comm_bytes(D, x, w);
      const Obj o = objective(D, w, cm, dur);
      if (!have || obj_less(o, best)) {
        best = o;
        bcomm = cm;
        have = true;
      }
    };
    if (mode <= 1) {
      for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
        const int w = rr.idx[i];
        if (run(w) && (mode == 1 || held(w))) consider(w);
      }
    } else if (mode <= 3) {
      for (int w = threadIdx.x; w < D.W; w += blockDim.x)
        if (run(w) && (mode == 3 || held(w))) consider(w);
    }
    ArgBest b = block_argmin(best, bcomm, have);
    if (threadIdx.x == 0) {
      if (b.o.w == INT32_MAX) {
        D.state[x] = S_NO_WORKER;
        atomicAdd((unsigned long long*)&D.g_relwait[D.group[x]], (unsigned long long)-1ll);
        c->n_unrunnable++;
      } else {
        place_eager(D, x, b.o.w, ROUTE_NONROOTISH, b.comm, stage_next, dur);
      }
    }
  } else {  // fast path over an ordered pool
    bool use_idle = c->n_idle > 0;
    int64_t n = gather_pool(D, use_idle, S.pool, 32);
    if (n == 0) {  // no running worker: no-worker (:2289-2290)
      if (threadIdx.x == 0) {
        D.state[x] = S_NO_WORKER;
        atomicAdd((unsigned long long*)&D.g_relwait[D.group[x]], (unsigned long long)-1ll);
        c->n_unrunnable++;
      }
    } else if (op == OP_KTH && n >= 20) {
      // pool[n_tasks % n] — n >= 20 idle workers: find the k-th idle worker
      int64_t k = c->n_tasks % n;
      int64_t base = 0;
      __shared__ int s_kth;
      for (int w0 = 0; w0 < D.W; w0 += blockDim.x) {
        int w = w0 + threadIdx.x;
        bool in = w < D.W && (use_idle ? (WK_flags(D)[w] & WF_IDLE) : !(WK_flags(D)[w] & WF_PAUSED));
        int64_t tot;
        int64_t pos = block_excl_scan(in ? 1 : 0, &tot);
        if (in && base + pos == k) s_kth = w;
        base += tot;
      }
      __syncthreads();
      if (threadIdx.x == 0) place_eager(D, x, s_kth, ROUTE_FASTPATH, -1, stage_next, dur);
    } else if (threadIdx.x == 0) {
      int best = S.pool[0];
      double bocc = occupancy(D, best, dur);
      for (int64_t i = 1; i < n; i++) {
        double o = occupancy(D, S.pool[i], dur);
        if (o < bocc) {
          best = S.pool[i];
          bocc = o;
        }
      }
      if (bocc == 0) {
        int64_t start = c->n_tasks % n;
        for (int64_t i = 0; i < n; i++) {
          int cand = S.pool[(i + start) % n];
          if (occupancy(D, cand, dur) == 0) {
            best = cand;
            break;
          }
        }
      }
      place_eager(D, x, best, ROUTE_FASTPATH, -1, stage_next, dur);
    }
  }
  __syncthreads();
}

// dispatch S.list[0..nlist) in order (all lanes)
__device__ __attribute__((noinline)) void dispatch_list_coop(const Dev& D, CoopShared& S, int64_t* stage_next, const double* dur) {
  if (threadIdx.x == 0) S.pos = 0;
  __syncthreads();
  while (true) {
    if (threadIdx.x == 0) {
      S.op = OP_NONE;
      while (S.pos < S.nlist) {
        int x = S.list[S.pos];
        int op = dispatch_prepare(D, x, S, stage_next, dur);
        if (op != OP_NONE) {
          S.op = op;
          S.x = x;
          break;
        }
        S.pos++;
      }
    }
    __syncthreads();
    if (S.op == OP_NONE) break;
    dispatch_collective(D, S, stage_next, dur);
    if (threadIdx.x == 0) S.pos++;
    __syncthreads();
  }
}

// Scheduler.stimulus_queue_slots_maybe_opened :4983-5023 (lane 0, tree maintained)
__device__ __attribute__((noinline)) void queue_refill_eager(const Dev& D, int64_t* stage_next, const double* dur) {
  Ctl* c = D.ctl;
  if (c->qlen == 0) return;
  int64_t slots = c->itc_slots;
  for (int64_t k = 0; k < slots; k++) {
    if (c->qlen == 0) return;
    if (c->n_itc == 0) continue;  // stays queued
    int q = D.qarr[c->qhead];
    c->qhead++;
    c->qlen--;
    place_eager(D, q, D.t_idx[1], ROUTE_ROOTISH_Q, -1, stage_next, dur);
  }
}

// resolve the queued tasks taken by local stimuli [from, to) (all lanes)
__device__ __attribute__((noinline)) void resolve_pops_coop(const Dev& D, const int32_t* L, int from, int to) {
  Ctl* c = D.ctl;
  int64_t base = 0;
  for (int j0 = from; j0 < to; j0 += blockDim.x) {
    int j = j0 + threadIdx.x;
    int64_t k = (j < to) ? D.ev_pops[j] : 0;
    int64_t tot;
    int64_t off = block_excl_scan(k, &tot);
    if (k > 0) {
      int w = D.ev_w[j];
      int64_t st0 = D.ev_plbase[j] + D.ev_npl[j] - k;
      for (int64_t i = 0; i < k; i++) {
        int q = D.qarr[c->qhead + base + off + i];
        D.st_task[st0 + i] = q;
        D.proc_on[q] = w;
        D.state[q] = S_PROCESSING;
      }
    }
    base += tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    c->qhead += base;
    c->qlen -= base;
    if (c->qlen < 0) set_error(D, ERR_QUEUE, -1);
  }
  __syncthreads();
}


// ================================================================== kernels

__global__ void k_init_workers(const Dev* __restrict__ Dp) {
  const Dev& D = *Dp;
  for (int w = blockIdx.x * blockDim.x + threadIdx.x; w < D.W; w += gridDim.x * blockDim.x) {
    WK_nproc(D)[w] = 0;
    WK_plen(D)[w] = 0;
    WK_netocc(D)[w] = 0;
    WK_nbytes(D)[w] = 0;
    WK_itcslots(D)[w] = 0;
    WK_lastcheck(D)[w] = ~0ull;
    for (int i = 0; i < NEEDS_W; i++) D.w_needs[(size_t)w * NEEDS_W + i] = 0;
    // Scheduler.add_worker ends with check_idle_saturated(ws) (:4418): a worker with no
    // tasks is idle (p < nthreads), never saturated, and in idle_task_count unless its
    // slot count is 0
    bool itc = !worker_full(D, w);
    WK_flags(D)[w] = WF_IDLE | (itc ? WF_ITC : 0);
    if (itc) {
      WK_itcslots(D)[w] = task_slots_available(D, w);
      atomicAdd((unsigned long long*)&D.ctl->n_itc, 1ull);
      atomicAdd((unsigned long long*)&D.ctl->itc_slots, (unsigned long long)WK_itcslots(D)[w]);
    }
    atomicAdd((unsigned long long*)&D.ctl->n_idle, 1ull);
  }
}

// update_graph, part 1 (:4600-4611 -> _transition_released_waiting :2078-2119), every
// task in parallel: waiting_on = dependencies without a replica; waiters = dependents
// (all of them go to waiting in the same stimulus; priorities are topological)
// (tasks [lo, N): lo = 0 for the first graph, the first new task for a later one)
// update_graph, part 1 (released -> waiting, :2078-2119): waiting_on = the dependencies not
// in memory, waiters = the dependents. Each wave takes 64 consecutive tasks, one per lane;
// a row wider than 32 dependencies (the P2P barrier's 66,666) is counted by the whole wave
// afterwards instead of one lane's serial loop.
__device__ __forceinline__ bool ug_dep_in_memory(const Dev& D, int d) {
  // every word loaded independently (no exit on the first set bit: the loads issue back to
  // back, one memory round trip per row instead of one per word)
  const unsigned long long* row = D.holders + (size_t)d * D.WB;
  unsigned long long any = 0;
  for (int wd = 0; wd < D.WB; wd++) any |= row[wd];
  return any != 0;
}
// a row wider than this is counted by k_ug_init_wide's grid (the host launches it for each
// such task, dgplace.hip launch_ug_init); k_ug_init leaves it at 0
constexpr int64_t UG_WIDE = 2048;
__global__ void k_ug_init(const Dev* __restrict__ Dp, int lo) {
  const Dev& D = *Dp;
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t t0 = lo + wave * 64; t0 < D.N; t0 += nwaves * 64) {
    const int64_t t = t0 + lane;
    const bool in = t < D.N;
    const int64_t a = in ? D.dep_ptr[t] : 0, b = in ? D.dep_ptr[t + 1] : 0;
    const bool wide = b - a > 32;
    if (in && !wide) {
      int wo = 0;
      for (int64_t k = a; k < b; k++) wo += ug_dep_in_memory(D, D.dep_idx[k]) ? 0 : 1;
      D.remaining[t] = wo;
      D.waiters[t] = (int32_t)(D.dpt_ptr[t + 1] - D.dpt_ptr[t]);
      D.state[t] = S_WAITING;
    }
    for (unsigned long long wm = __ballot(wide); wm; wm &= wm - 1) {
      const int j = __builtin_ctzll(wm);
      const int64_t tw = t0 + j;
      const int64_t aw = __shfl(a, j), bw = __shfl(b, j);
      int64_t wo = 0;
      if (bw - aw <= UG_WIDE)
        for (int64_t k = aw + lane; k < bw; k += 64) wo += ug_dep_in_memory(D, D.dep_idx[k]) ? 0 : 1;
      wo = wave_sum64(wo);
      if (lane == 0) {
        D.remaining[tw] = (int32_t)wo;
        D.waiters[tw] = (int32_t)(D.dpt_ptr[tw + 1] - D.dpt_ptr[tw]);
        D.state[tw] = S_WAITING;
      }
    }
  }
}

// the dependencies not in memory of one row wider than UG_WIDE (the P2P barrier's 66,666),
// over the whole grid: k_ug_init left remaining[t] at 0 and this adds each block's count
__global__ void k_ug_init_wide(const Dev* __restrict__ Dp, int t, int64_t a, int64_t b) {
  const Dev& D = *Dp;
  int cnt = 0;
  for (int64_t k = a + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < b; k += (int64_t)gridDim.x * blockDim.x)
    cnt += ug_dep_in_memory(D, D.dep_idx[k]) ? 0 : 1;
  cnt = (int)wave_sum64(cnt);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&D.remaining[t], cnt);
}

// update_graph's ready list (the tasks of order[scan_lo, N) from task_lo on with no
// remaining dependency, in priority order) over many workgroups: each takes a tile of
// RDY_TILE order entries, counts its ready tasks (k_ready_count), then writes them at the
// sum of the earlier tiles' counts (k_ready_scatter); the last tile writes the total, which
// k_ug_dispatch takes as its list length
constexpr int RDY_TILE = 4 * CTA;
__global__ void __launch_bounds__(CTA) k_ready_count(const Dev* __restrict__ Dp, int scan_lo, int task_lo, int64_t* cnt) {
  const Dev& D = *Dp;
  const int64_t base = scan_lo + (int64_t)blockIdx.x * RDY_TILE;
  int c = 0;
  for (int j = 0; j < RDY_TILE / CTA; j++) {
    const int64_t i = base + (int64_t)j * CTA + threadIdx.x;
    const int t = i < D.N ? D.order[i] : -1;
    c += (t >= task_lo && D.remaining[t] == 0) ? 1 : 0;
  }
  int64_t tot;
  block_excl_scan(c, &tot);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}
__global__ void __launch_bounds__(CTA) k_ready_scatter(const Dev* __restrict__ Dp, int scan_lo, int task_lo,
                                                       const int64_t* cnt, int64_t* total) {
  const Dev& D = *Dp;
  int64_t off = 0;
  for (int k = threadIdx.x; k < (int)blockIdx.x; k += CTA) off += cnt[k];
  int64_t off_tot;
  block_excl_scan(off, &off_tot);
  const int64_t base = scan_lo + (int64_t)blockIdx.x * RDY_TILE;
  int64_t run = off_tot;
  for (int j = 0; j < RDY_TILE / CTA; j++) {
    const int64_t i = base + (int64_t)j * CTA + threadIdx.x;
    const int t = i < D.N ? D.order[i] : -1;
    const bool r = t >= task_lo && D.remaining[t] == 0;
    int64_t tot;
    const int64_t pos = block_excl_scan(r ? 1 : 0, &tot);
    if (r) D.ready[run + pos] = t;
    run += tot;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *total = run;
}

// k_ug_dispatch's dynamic LDS: the tournament tree and the worker arrays its lane-0 chain of
// dependent reads and writes walks per placement, staged in LDS when they fit (bit k of
// `mask`: array k, in this order; the host picks the prefix that fits its LDS budget). The
// dispatch's LDS copy of Dev points at the staged copies, so every callee uses them as is.
constexpr int UG_NF = 15;
__host__ __device__ inline size_t ug_field_bytes(int k, int W, int Wp, int P) {
  switch (k) {
    case 13: case 14: return (size_t)P * sizeof(double);  // pdur_cur, pdur_walk
    case 0: return 2 * (size_t)Wp * sizeof(double);   // t_key
    case 1: return 2 * (size_t)Wp * sizeof(int32_t);  // t_idx
    case 2: case 3: case 4: case 5: return (size_t)W * 4;  // nproc, nthreads, cap, plen
    case 6: return (size_t)W;                                  // flags
    case 7: case 8: case 9: case 10: return (size_t)W * 8;     // itcslots, netocc, nbytes, lastcheck
    default: return (size_t)W * PMAX * 4;                      // pfx, pcnt
  }
}
__host__ __device__ inline size_t ug_field_off(int k, int W, int Wp, int P, uint32_t mask) {  // 16-aligned
  size_t o = 0;
  for (int j = 0; j < k; j++)
    if (mask >> j & 1) o += (ug_field_bytes(j, W, Wp, P) + 15) & ~(size_t)15;
  return o;
}
__device__ inline void** ug_field_ptr(Dev& d, int k) {
  switch (k) {
    case 0: return (void**)&d.t_key;
    case 1: return (void**)&d.t_idx;
    case 2: return (void**)&d.w_nproc;
    case 3: return (void**)&d.w_nthreads;
    case 4: return (void**)&d.w_cap;
    case 5: return (void**)&d.w_plen;
    case 6: return (void**)&d.w_flags;
    case 7: return (void**)&d.w_itcslots;
    case 8: return (void**)&d.w_netocc;
    case 9: return (void**)&d.w_nbytes;
    case 10: return (void**)&d.w_lastcheck;
    case 11: return (void**)&d.w_pfx;
    case 12: return (void**)&d.w_pcnt;
    case 13: return (void**)&d.pdur_cur;
    default: return (void**)&d.pdur_walk;
  }
}
// dir 0: global -> LDS (and the Dev copy points at LDS); 1: LDS -> global (g: the global Dev)
__device__ inline void ug_stage(Dev& d, const Dev& g, uint32_t mask, int dir) {
  for (int k = 0; k < UG_NF; k++) {
    if (!(mask >> k & 1)) continue;
    const size_t nb = ug_field_bytes(k, d.W, d.Wp, d.P);
    char* l = dgp_smem + ug_field_off(k, d.W, d.Wp, d.P, mask);
    char* gp = (char*)*ug_field_ptr(const_cast<Dev&>(g), k);
    char* src = dir == 0 ? gp : l;
    char* dst = dir == 0 ? l : gp;
    const size_t nw = nb / 4;
    for (size_t i = threadIdx.x; i < nw; i += blockDim.x) ((uint32_t*)dst)[i] = ((const uint32_t*)src)[i];
    for (size_t i = nw * 4 + threadIdx.x; i < nb; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  if (dir == 0 && threadIdx.x == 0)
    for (int k = 0; k < UG_NF; k++)
      if (mask >> k & 1) *ug_field_ptr(d, k) = dgp_smem + ug_field_off(k, d.W, d.Wp, d.P, mask);
  __syncthreads();
}

// update_graph's root-ish dispatch with queuing (decide_worker_rootish_queuing_enabled
// :2195-2245, then _add_to_processing :3199-3256 as place_eager does it) for a run of
// consecutive dependency-free root-ish ready tasks of one prefix, every pick at once.
// The pick is the idle_task_count worker of least len(processing) / nthreads (ties: the
// canonical index); a pick changes only the picked worker's count. With one nthreads over
// idle_task_count the picks are therefore the pairs (v, m) -- worker v at processing count
// m, nproc_v <= m < nproc_v + slots_v -- in ascending (m, v) order: pair (v, m)'s rank is
// the pairs of the levels below m plus the workers before v at level m, and pick r takes
// ready[pos + r]. For such tasks (no comm bytes, no needs_what, one prefix p) everything
// place_eager does at pick r on v (the k-th on v) is a function of (v, k, r) and the state
// before the run: v's dict with p counted k (+1 after), nproc_v + k, the global dict with p
// counted r + 1 (total_occupancy for check_idle_saturated's idle / saturated test). So the
// picks are one thread each, the workers' end states (dict, nproc, idle / saturated of
// their last pick, idle_task_count) one thread per worker, and the tree is rebuilt after.
// All threads; returns the picks made, 0 when the run does not qualify (the serial path
// takes the task and raises any capacity error as before).
constexpr int UG_FILL_LEVELS = 64;
__device__ __attribute__((noinline)) int64_t ug_fill_rootish(const Dev& D, int64_t pos, int64_t nr, int64_t stage0,
                                                             const double* dur) {
  __shared__ int64_t f_lvl[UG_FILL_LEVELS + 1];  // pairs below each level (exclusive prefix)
  __shared__ int f_ok, f_nth, f_mlo, f_mhi, f_run;
  __shared__ int64_t f_stot, f_M;
  Ctl* c = D.ctl;
  const int tid = threadIdx.x;
  const int x0 = D.ready[pos];
  const int p = D.prefix[x0];
  if (tid == 0) {
    f_ok = (D.tflags[x0] & TF_ROOTISH) && D.dep_ptr[x0 + 1] == D.dep_ptr[x0] && p >= 0 && p < D.P ? 1 : 0;
    f_nth = -1;
    f_mlo = INT32_MAX;
    f_mhi = -1;
    f_run = INT32_MAX;
    f_stot = 0;
  }
  __syncthreads();
  if (!f_ok) return 0;
  // the run: consecutive ready tasks from pos that are root-ish, dependency-free, of prefix p
  for (int64_t i0 = pos; i0 < nr && f_run == INT32_MAX; i0 += blockDim.x) {
    const int64_t i = i0 + tid;
    if (i < nr) {
      const int x = D.ready[i];
      if (!((D.tflags[x] & TF_ROOTISH) && D.dep_ptr[x + 1] == D.dep_ptr[x] && D.prefix[x] == p))
        atomicMin(&f_run, (int)(i - pos));
    }
    __syncthreads();
  }
  const int64_t M = f_run == INT32_MAX ? nr - pos : (int64_t)f_run;
  // idle_task_count: one nthreads, the level span, the slots; every picked worker's dict
  // must hold p or have room for it (else the serial path raises ERR_PREFIX_CAP)
  for (int v = tid; v < D.W; v += blockDim.x) {
    if (!(WK_flags(D)[v] & WF_ITC)) continue;
    const int nt = WK_nthreads(D)[v];
    const int np = WK_nproc(D)[v];
    const int64_t sl = task_slots_available(D, v);
    if (sl <= 0 || nt <= 0) {
      f_ok = 0;
      continue;
    }
    if (atomicCAS(&f_nth, -1, nt) != -1 && f_nth != nt) f_ok = 0;
    atomicMin(&f_mlo, np);
    atomicMax(&f_mhi, (int)(np + sl - 1));
    atomicAdd((unsigned long long*)&f_stot, (unsigned long long)sl);
    const int n = WK_plen(D)[v];
    bool has = false;
    for (int i = 0; i < n; i++) has = has || WK_pfx(D)[(size_t)v * PMAX + i] == p;
    if (!has && n >= PMAX) f_ok = 0;
  }
  __syncthreads();
  if (!f_ok || f_nth <= 0 || f_stot <= 0 || f_mhi - f_mlo + 1 > UG_FILL_LEVELS) return 0;
  const int64_t Mp = M < f_stot ? M : f_stot;
  bool gdict_room = false;
  for (int i = 0; i < c->g_plen; i++) gdict_room = gdict_room || c->g_pfx[i] == p;
  if ((!gdict_room && c->g_plen >= PMAX_G) || stage0 + Mp > D.st_cap) return 0;
  const int mlo = f_mlo, L = f_mhi - f_mlo + 1;
  // pairs per level, then their exclusive prefix over the levels
  if (tid <= L) f_lvl[tid] = 0;
  __syncthreads();
  for (int v = tid; v < D.W; v += blockDim.x) {
    if (!(WK_flags(D)[v] & WF_ITC)) continue;
    const int np = WK_nproc(D)[v];
    const int64_t sl = task_slots_available(D, v);
    for (int64_t k = 0; k < sl; k++) atomicAdd((unsigned long long*)&f_lvl[np + k - mlo + 1], 1ull);
  }
  __syncthreads();
  if (tid == 0)
    for (int l = 1; l <= L; l++) f_lvl[l] += f_lvl[l - 1];
  __syncthreads();
  // ranks: per level, the workers in index order (a block scan over the workers); pick r of
  // worker v (its k-th) records v in the staging row and k in st_comm (0 once placed)
  // scratch (the tree is rebuilt after): each worker's last pick, its rank and its k
  int32_t* last = D.t_idx;
  double* last_k = D.t_key;
  for (int v = tid; v < D.W; v += blockDim.x) last[v] = -1;
  __syncthreads();
  for (int l = 0; l < L; l++) {
    const int m = mlo + l;
    if (f_lvl[l] >= Mp) break;
    int64_t base = 0;
    for (int v0 = 0; v0 < D.W; v0 += blockDim.x) {
      const int v = v0 + tid;
      bool in = false;
      if (v < D.W && (WK_flags(D)[v] & WF_ITC)) {
        const int np = WK_nproc(D)[v];
        in = np <= m && m < np + task_slots_available(D, v);
      }
      int64_t tot;
      const int64_t o = block_excl_scan(in ? 1 : 0, &tot);
      const int64_t r = f_lvl[l] + base + o;
      if (in && r < Mp) {
        D.st_worker[stage0 + r] = v;
        D.st_comm[stage0 + r] = m - WK_nproc(D)[v];
        last[v] = (int32_t)r;  // levels ascend: the last level written is the worker's last pick
        last_k[v] = (double)(m - WK_nproc(D)[v]);
      }
      base += tot;
    }
  }
  __syncthreads();
  __threadfence_block();
  // the picks, one thread each: the placement record (worker_objective's start before the
  // pick, ws.nbytes) and the task's TaskState
  const double bw = (double)D.bandwidth;
  auto occ_k = [&](int v, int64_t k) {  // v's occupancy with p counted k more times (:1884-1903)
    double res = 0.0;
    const int n = WK_plen(D)[v];
    const int* pf = WK_pfx(D) + (size_t)v * PMAX;
    const int* pc = WK_pcnt(D) + (size_t)v * PMAX;
    bool has = false;
    for (int i = 0; i < n; i++) {
      const int64_t cnt = pc[i] + (pf[i] == p ? k : 0);
      has = has || pf[i] == p;
      res += prefix_duration(D, dur, pf[i]) * (double)cnt;
    }
    if (!has && k > 0) res += prefix_duration(D, dur, p) * (double)k;  // appended at the first pick
    return res + (double)WK_netocc(D)[v] / bw;
  };
  for (int64_t r = tid; r < Mp; r += blockDim.x) {
    const int v = D.st_worker[stage0 + r];
    const int64_t k = D.st_comm[stage0 + r];
    const int x = D.ready[pos + r];
    const double stack = occ_k(v, k) / (double)WK_nthreads(D)[v];
    D.st_task[stage0 + r] = x;
    D.st_comm[stage0 + r] = 0;
    D.st_start[stage0 + r] = stack + (double)0 / bw;
    D.st_wsnbytes[stage0 + r] = WK_nbytes(D)[v];
    D.st_route[stage0 + r] = (int8_t)ROUTE_ROOTISH_Q;
    D.proc_on[x] = v;
    if (D.state[x] == S_WAITING) atomicAdd((unsigned long long*)&D.g_relwait[D.group[x]], (unsigned long long)-1ll);
    D.state[x] = S_PROCESSING;
  }
  // total_occupancy after pick r (the global dict with p counted r + 1 more, :1877)
  int gi = -1;
  for (int i = 0; i < c->g_plen; i++)
    if (c->g_pfx[i] == p) gi = i;
  auto total_occ = [&](int64_t r) {
    double res = 0.0;
    for (int i = 0; i < c->g_plen; i++)
      res += prefix_duration(D, D.pdur_walk, c->g_pfx[i]) * (double)(c->g_pcnt[i] + (i == gi ? r + 1 : 0));
    if (gi < 0) res += prefix_duration(D, D.pdur_walk, p) * (double)(r + 1);
    return res + c->g_netocc / bw;
  };
  __syncthreads();
  // the workers' end states, one thread each: check_idle_saturated of its last pick
  // (walk_flags' rule), its dict / nproc, then idle_task_count (itc_check without the tree)
  __shared__ long long f_didle, f_dsat, f_ditc, f_dslots;
  if (tid == 0) f_didle = f_dsat = f_ditc = f_dslots = 0;
  __syncthreads();
  for (int v = tid; v < D.W; v += blockDim.x) {
    const int32_t rl = last[v];
    if (rl < 0) continue;
    const int64_t npk = (int64_t)last_k[v] + 1;  // its picks: k = 0 .. the last one's
    // dict and nproc after npk picks of prefix p (wdict_inc's append on the first)
    int* pf = WK_pfx(D) + (size_t)v * PMAX;
    int* pc = WK_pcnt(D) + (size_t)v * PMAX;
    const int n = WK_plen(D)[v];
    int hi = -1;
    for (int i = 0; i < n; i++)
      if (pf[i] == p) hi = i;
    if (hi >= 0) {
      pc[hi] += (int)npk;
    } else {
      pf[n] = p;
      pc[n] = (int)npk;
      WK_plen(D)[v] = n + 1;
    }
    WK_nproc(D)[v] += (int32_t)npk;
    // idle / saturated of the last pick (walk_flags, with total_occupancy after pick rl)
    {
      const int64_t pn = WK_nproc(D)[v];
      const int64_t nt = WK_nthreads(D)[v];
      const uint8_t fl = WK_flags(D)[v];
      const double occ = occ_k(v, 0);
      bool idle = false, sat = false;
      double avg = -1;
      if (fl & WF_PAUSED) {
      } else if (pn < nt) {
        idle = true;
      } else {
        avg = total_occ(rl) / (double)D.total_nthreads;
        idle = occ < (double)nt * avg / 2;
      }
      if (!idle && pn > nt && !(fl & WF_PAUSED)) {
        const double pending = occ * (double)(pn - nt) / (double)(pn * nt);
        if (0.4 < pending) {
          if (avg < 0) avg = total_occ(rl) / (double)D.total_nthreads;
          sat = pending > 1.9 * avg;
        }
      }
      if (idle != ((fl & WF_IDLE) != 0)) atomicAdd((unsigned long long*)&f_didle, idle ? 1ull : (unsigned long long)-1ll);
      if (sat != ((fl & WF_SAT) != 0)) atomicAdd((unsigned long long*)&f_dsat, sat ? 1ull : (unsigned long long)-1ll);
      uint8_t nf = (fl & ~(WF_IDLE | WF_SAT)) | (idle ? WF_IDLE : 0) | (sat ? WF_SAT : 0);
      // idle_task_count (itc_check)
      const bool on = !worker_full(D, v) && !(nf & WF_PAUSED);
      if (on != ((nf & WF_ITC) != 0)) {
        nf = on ? (nf | WF_ITC) : (nf & ~WF_ITC);
        atomicAdd((unsigned long long*)&f_ditc, on ? 1ull : (unsigned long long)-1ll);
      }
      const int64_t contrib = on ? task_slots_available(D, v) : 0;
      const int64_t delta = contrib - WK_itcslots(D)[v];
      if (delta) atomicAdd((unsigned long long*)&f_dslots, (unsigned long long)delta);
      WK_itcslots(D)[v] = contrib;
      WK_flags(D)[v] = nf;
    }
  }
  __syncthreads();
  if (tid == 0) {
    c->n_idle += f_didle;
    c->n_sat += f_dsat;
    c->n_itc += f_ditc;
    c->itc_slots += f_dslots;
    c->n_tasks += Mp;
    if (gi >= 0) {
      c->g_pcnt[gi] += Mp;
    } else {
      c->g_pfx[c->g_plen] = p;
      c->g_pcnt[c->g_plen] = Mp;
      c->g_plen++;
    }
  }
  __threadfence_block();
  __syncthreads();
  tree_rebuild_coop(D);
  return Mp;
}

// update_graph, part 2: the tasks that went waiting -> processing, in priority order,
// dispatched one by one (they read global state); once idle_task_count is empty every
// further root-ish task is queued in bulk (:2761) — order-preserving.
// Tasks at priority positions [lo, N) (a later graph's tasks follow every earlier one in
// priority: a new generation); its placements append to the placement log.
// scan_lo: the first priority position scanned; task_lo: the first task of the graph (a later
// graph whose user priority outranks earlier tasks: its tasks sit anywhere in the order)
__global__ void __launch_bounds__(CTA) k_ug_dispatch(const Dev* __restrict__ Dp, const int64_t* __restrict__ ready_n,
                                                     int task_lo, uint32_t lds_mask) {
  // the dispatch is one lane's chain of dependent reads and writes of the control block
  // (idle_task_count / idle / saturated counts, the global prefix dict, occupancy sums): the
  // block works on an LDS copy of it (and of Dev, whose ctl points at the copy) and writes
  // it back at the end
  __shared__ Dev s_dev;
  __shared__ Ctl s_ctl;
  {
    static_assert(sizeof(Dev) % 4 == 0 && sizeof(Ctl) % 4 == 0, "word copies");
    const uint32_t* sd = (const uint32_t*)Dp;
    const uint32_t* sc = (const uint32_t*)Dp->ctl;
    for (int i = threadIdx.x; i < (int)(sizeof(Dev) / 4); i += blockDim.x) ((uint32_t*)&s_dev)[i] = sd[i];
    for (int i = threadIdx.x; i < (int)(sizeof(Ctl) / 4); i += blockDim.x) ((uint32_t*)&s_ctl)[i] = sc[i];
    __syncthreads();
    if (threadIdx.x == 0) s_dev.ctl = &s_ctl;
    __syncthreads();
    if (lds_mask) ug_stage(s_dev, *Dp, lds_mask, 0);
  }
  Ctl* const ctl_g = Dp->ctl;
  const Dev& D = s_dev;
  __shared__ CoopShared S;
  __shared__ int64_t s_nr, s_pos;
  Ctl* c = D.ctl;
  const int64_t pl0 = (int64_t)c->n_placed;  // 0 for the first graph
  // the ready list in priority order: D.ready[0, *ready_n) (k_ready_count / k_ready_scatter)
  (void)task_lo;
  if (threadIdx.x == 0) {
    s_nr = *ready_n;
    s_pos = 0;
  }
  tree_rebuild_coop(D);
  int64_t stage_next = 0;  // lane 0's overflow staging cursor
  const double* dur = D.pdur_cur;
  bool bulk_done = false;
  while (true) {
    __syncthreads();
    int64_t pos = s_pos, nr = s_nr;
    if (pos >= nr) break;
    // bulk queueing once idle_task_count is empty (saturation finite)
    if (!bulk_done && !D.sat_inf && c->n_itc == 0) {
      int64_t qb = c->qhead + c->qlen, kept = 0, queued = 0;
      for (int64_t i0 = pos; i0 < nr; i0 += blockDim.x) {
        int64_t i = i0 + threadIdx.x;
        int x = i < nr ? D.ready[i] : -1;
        bool q = x >= 0 && (D.tflags[x] & TF_ROOTISH);
        bool k = x >= 0 && !q;
        int64_t tq, tk;
        int64_t oq = block_excl_scan(q ? 1 : 0, &tq);
        int64_t ok = block_excl_scan(k ? 1 : 0, &tk);
        if (q) {
          D.qarr[qb + queued + oq] = x;
          D.state[x] = S_QUEUED;
        }
        // released + waiting of each queued task's group, one atomic per group a wave holds
        // (a root-ish run is mostly one group: per-task atomics on one address serialised)
        {
          const int g = q ? D.group[x] : -1;
          for (unsigned long long m = __ballot(q); m;) {
            const int g0 = __shfl(g, __builtin_ctzll(m));
            const unsigned long long mg = __ballot(q && g == g0);
            if ((threadIdx.x & 63) == __builtin_ctzll(m))
              atomicAdd((unsigned long long*)&D.g_relwait[g0], (unsigned long long)-(long long)__builtin_popcountll(mg));
            m &= ~mg;
          }
        }
        if (k) D.ready[pos + kept + ok] = x;
        queued += tq;
        kept += tk;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        c->qlen += queued;
        s_nr = pos + kept;
      }
      bulk_done = true;
      continue;
    }
    // a run of root-ish tasks while idle_task_count has room: every pick at once
    if (!D.sat_inf && c->n_itc > 0 && (D.tflags[D.ready[pos]] & TF_ROOTISH)) {
      __shared__ int64_t s_stage;
      if (threadIdx.x == 0) s_stage = stage_next;
      __syncthreads();
      const int64_t nf = ug_fill_rootish(D, pos, nr, s_stage, dur);
      if (nf > 0) {
        if (threadIdx.x == 0) {
          stage_next += nf;
          s_pos = pos + nf;
        }
        continue;
      }
    }
    int64_t chunk = nr - pos < FL_MAX ? nr - pos : FL_MAX;
    // stop the chunk at the point where the bulk path takes over
    if (threadIdx.x == 0) S.nlist = (int)chunk;
    for (int64_t i = threadIdx.x; i < chunk; i += blockDim.x) S.list[i] = D.ready[pos + i];  // every lane
    __syncthreads();
    if (threadIdx.x == 0) S.pos = 0;
    __syncthreads();
    while (true) {
      if (threadIdx.x == 0) {
        S.op = OP_NONE;
        S.done = 0;
        while (S.pos < S.nlist) {
          int x = S.list[S.pos];
          if (!bulk_done && !D.sat_inf && (D.tflags[x] & TF_ROOTISH) && c->n_itc == 0) {
            S.done = 1;  // hand the rest to the bulk path
            break;
          }
          int op = dispatch_prepare(D, x, S, &stage_next, dur);
          if (op != OP_NONE) {
            S.op = op;
            S.x = x;
            break;
          }
          S.pos++;
        }
      }
      __syncthreads();
      if (S.op == OP_NONE) break;
      dispatch_collective(D, S, &stage_next, dur);
      if (threadIdx.x == 0) S.pos++;
      __syncthreads();
    }
    if (threadIdx.x == 0) s_pos = pos + S.pos;
  }
  __syncthreads();
  // the stimulus' placements become the placement log head (run_id order)
  __shared__ int64_t s_np;
  if (threadIdx.x == 0) s_np = stage_next;
  __syncthreads();
  int64_t np = s_np;
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
    c->round_start = 0;
    c->round_n = 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < (int)(sizeof(Ctl) / 4); i += blockDim.x) ((uint32_t*)ctl_g)[i] = ((const uint32_t*)&s_ctl)[i];
  if (lds_mask) ug_stage(s_dev, *Dp, lds_mask, 1);
}

// start of a round: its completion list is the slice of the placement log made by the
// previous stimulus batch
__device__ void round_begin(const Dev& D, long long* next_start, const int32_t* ext, long long ext_n) {
  Ctl* c = D.ctl;
  if (ext) {  // an explicit batch of completions (dgp_tasks_finished)
    c->round_L = ext;
    c->round_n = ext_n;
    *next_start = (long long)c->n_placed;
  } else {
    c->round_L = D.pl_task + *next_start;
    c->round_n = (long long)c->n_placed - *next_start;
    *next_start = (long long)c->n_placed;
  }
  c->n_frontier = 0;
  c->pool_used = 0;
  c->round_counter++;
  if (c->round_n > 0) c->rounds_nonempty++;
}
__global__ void k_round_begin(const Dev* __restrict__ Dp, long long* next_start, const int32_t* ext, long long ext_n) {
  round_begin(*Dp, next_start, ext, ext_n);
}

__device__ void frontier_release_body(const Dev& D, int64_t gtid, int64_t gthreads) {
  const Ctl* c = D.ctl;
  const int64_t n = c->round_n;
  const int32_t* L = c->round_L;
  const unsigned long long tag = (unsigned long long)c->round_counter << 32;
  for (int64_t j = gtid; j < n; j += gthreads) {
    int t = L[j];
    unsigned long long key = tag | (unsigned long long)j;
    // the replica this completion creates is known before the ordered commit: publish it
    // now (who_has bit, set_nbytes) so k_candidate_commbytes sees it. Only t's dependents
    // read it, and they become ready at j or later.
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

__global__ void k_frontier_release(const Dev* __restrict__ Dp) {
  frontier_release_body(*Dp, blockIdx.x * (int64_t)blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

// one wave per newly ready task: candidate workers (OR of the dependencies' replica
// bitsets) and, per candidate, the exact comm bytes (total minus what it holds)
// one wave: task x's candidates (pool entries from ctl->pool_used on)
__device__ void candidate_row(const Dev& D, int x) {
  const int lane = threadIdx.x & 63;
  {
    int64_t d0 = D.dep_ptr[x], d1 = D.dep_ptr[x + 1];
    if (d1 == d0 || (D.tflags[x] & TF_ROOTISH) || restricted_nonrootish(D, x)) {
      if (lane == 0) D.cand_n[x] = 0;
      return;
    }
    int64_t tot = 0;
    for (int64_t k = d0 + lane; k < d1; k += 64) tot += get_nbytes(D, D.dep_idx[k]);
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
    // candidates = who_has of the dependencies & running (a paused worker is not valid,
    // decide_worker_non_rootish :2262-2266)
    auto running_bits = [&](int wd) {
      unsigned long long m = 0;
      if (D.evf & EVF_PAUSED)
        for (int b = 0; b < 64 && wd * 64 + b < D.W; b++) m |= (WK_flags(D)[wd * 64 + b] & WF_PAUSED) ? 1ull << b : 0ull;
      return ~m;
    };
    int total_c = 0;
    for (int wd0 = 0; wd0 < D.WB; wd0 += 64) {
      int wd = wd0 + lane;
      unsigned long long acc = 0;
      if (wd < D.WB) {
        for (int64_t k = d0; k < d1; k++) acc |= D.holders[(size_t)D.dep_idx[k] * D.WB + wd];
        acc &= running_bits(wd);
      }
      int cnt = __popcll(acc);
      for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
      total_c += cnt;
    }
    int64_t base = 0;
    if (lane == 0) {
      base = (int64_t)atomicAdd(&D.ctl->pool_used, (unsigned long long)total_c);
      if (base + total_c > D.pool_cap) set_error(D, ERR_POOL, x);
    }
    base = __shfl(base, 0);
    if (base + total_c > D.pool_cap) return;
    int64_t pos = base;
    for (int wd0 = 0; wd0 < D.WB; wd0 += 64) {
      int wd = wd0 + lane;
      unsigned long long acc = 0;
      if (wd < D.WB) {
        for (int64_t k = d0; k < d1; k++) acc |= D.holders[(size_t)D.dep_idx[k] * D.WB + wd];
        acc &= running_bits(wd);
      }
      int cnt = __popcll(acc);
      int incl = cnt;
      for (int o = 1; o < 64; o <<= 1) {
        int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      int64_t p = pos + incl - cnt;
      while (acc) {
        int b = __ffsll((long long)acc) - 1;
        acc &= acc - 1;
        D.pool_w[p++] = wd * 64 + b;
      }
      pos += __shfl(incl, 63);
    }
    for (int ci = lane; ci < total_c; ci += 64) {
      int cw = D.pool_w[base + ci];
      int64_t held = 0;
      for (int64_t k = d0; k < d1; k++) {
        int d = D.dep_idx[k];
        if (holds(D, d, cw)) held += get_nbytes(D, d);
      }
      D.pool_comm[base + ci] = tot - held;
    }
    if (lane == 0) {
      D.cand_off[x] = base;
      D.cand_n[x] = total_c;
    }
  }
}
__device__ void candidate_body(const Dev& D, int64_t wave, int64_t nwaves) {
  const int64_t nF = (int64_t)D.ctl->n_frontier;
  for (int64_t i = wave; i < nF; i += nwaves) candidate_row(D, D.frontier[i]);
}

__global__ void k_candidate_commbytes(const Dev* __restrict__ Dp) {
  candidate_body(*Dp, (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6, ((int64_t)gridDim.x * blockDim.x) >> 6);
}

enum : uint8_t { EV_MAYQUEUE = 2 };

// per completion stimulus j: the workers it may touch and whether it reads global state
__device__ void events_body(const Dev& D, int64_t gtid, int64_t gthreads) {
  const Ctl* c = D.ctl;
  const int64_t n = c->round_n;
  const int32_t* L = c->round_L;
  const unsigned long long tag = (unsigned long long)c->round_counter << 32;
  for (int64_t j = gtid; j < n; j += gthreads) {
    int t = L[j];
    unsigned long long key = tag | (unsigned long long)j;
    int w = D.proc_on[t];
    int32_t* touch = D.ev_touch + (size_t)j * TOUCH_MAX;
    int nt = 0;
    uint8_t fl = 0;
    auto add = [&](int x) {
      for (int i = 0; i < nt; i++)
        if (touch[i] == x) return;
      if (nt < TOUCH_MAX)
        touch[nt++] = x;
      else
        fl |= EV_GLOBAL;
    };
    add(w);
    for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
      int d = D.dep_idx[k];
      if (D.release_key[d] == key && D.waiters[d] == 0 && !(D.tflags[d] & TF_WANTED)) {
        const unsigned long long* row = D.holders + (size_t)d * D.WB;
        for (int wd = 0; wd < D.WB; wd++) {
          unsigned long long bits = row[wd];
          while (bits) {
            int b = __ffsll((long long)bits) - 1;
            bits &= bits - 1;
            add(wd * 64 + b);
          }
        }
      }
    }
    int nf = 0;
    // the one-wave local executor handles <= 64 dependencies / dependents / candidates
    // and <= 8 released tasks per stimulus; anything bigger runs as a global stimulus
    if (D.dep_ptr[t + 1] - D.dep_ptr[t] > 64 || D.dpt_ptr[t + 1] - D.dpt_ptr[t] > 64) fl |= EV_GLOBAL;
    for (int64_t k = D.dpt_ptr[t]; k < D.dpt_ptr[t + 1]; k++) {
      int x = D.dpt_idx[k];
      if (!is_frontier(D, x, key)) continue;
      nf++;
      if (D.tflags[x] & TF_ROOTISH) {
        fl |= EV_GLOBAL | (D.sat_inf ? 0 : EV_MAYQUEUE);
      } else if (D.dep_ptr[x + 1] == D.dep_ptr[x] || restricted_nonrootish(D, x)) {
        fl |= EV_GLOBAL;
      } else {
        int cn = D.cand_n[x];
        int64_t off = D.cand_off[x];
        if (cn > 64 || D.dep_ptr[x + 1] - D.dep_ptr[x] > 64) fl |= EV_GLOBAL;
        for (int i = 0; i < cn && i < 64; i++) add(D.pool_w[off + i]);
      }
    }
    if (nf > 8) fl |= EV_GLOBAL;
    D.ev_w[j] = w;
    D.ev_nf[j] = nf;
    D.ev_flags[j] = fl;
    D.ev_ntouch[j] = nt;
  }
}
__global__ void k_events(const Dev* __restrict__ Dp) {
  events_body(*Dp, blockIdx.x * (int64_t)blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

// global stimulus j (all lanes): waits for nothing — every earlier stimulus has committed
__device__ __attribute__((noinline)) void exec_global(const Dev& D, const int32_t* L, int j, unsigned long long key, const double* dur,
                            CoopShared& S, int64_t* stage_next, int* resolved_upto) {
  Ctl* c = D.ctl;
  resolve_pops_coop(D, L, *resolved_upto, j);
  if (threadIdx.x == 0) {
    *resolved_upto = j;
    unsigned long long tw = __builtin_amdgcn_s_memtime();
    walk_to(D, (unsigned long long)D.ev_recbase[j]);
    (void)tw;
  }
  __syncthreads();
  tree_rebuild_coop(D);
  __shared__ int64_t s_st0;
  __shared__ int64_t s_dpos;
  int t = L[j];
  if (threadIdx.x == 0) {
    s_st0 = *stage_next;
    int w = D.proc_on[t];
    int p = D.prefix[t];
    D.proc_on[t] = -1;
    wdict_dec(D, w, p);
    WK_nproc(D)[w]--;
    int64_t dnet = 0;
    if (D.dep_ptr[t + 1] > D.dep_ptr[t]) {
      for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) dnet -= needs_dec(D, w, D.dep_idx[k], t);
      WK_netocc(D)[w] += dnet;
    }
    needs_maybe_reset(D, w);
    apply_now(D, REC_COMPLETE, t, w, p, dnet, dur);
    itc_check(D, w, true);
    WK_nbytes(D)[w] += get_nbytes(D, t);
    D.state[t] = S_MEMORY;
    do_releases(D, t, key);
    s_dpos = D.dpt_ptr[t];
    c->n_global_events++;
  }
  __syncthreads();
  // frontier in ascending priority, in chunks of FL_MAX
  while (true) {
    if (threadIdx.x == 0) {
      S.nlist = 0;
      int64_t k = s_dpos;
      for (; k < D.dpt_ptr[t + 1] && S.nlist < FL_MAX; k++) {
        int x = D.dpt_idx[k];
        if (is_frontier(D, x, key)) S.list[S.nlist++] = x;
      }
      s_dpos = k;
    }
    __syncthreads();
    if (S.nlist == 0) break;
    dispatch_list_coop(D, S, stage_next, dur);
  }
  if (threadIdx.x == 0) {
    queue_refill_eager(D, stage_next, dur);
    D.ev_plbase[j] = s_st0;
    D.ev_npl[j] = (int32_t)(*stage_next - s_st0);
    D.ev_pops[j] = 0;
    *resolved_upto = j + 1;
  }
  __syncthreads();
}

// bytes of dynamic LDS per worker when the commit keeps worker state on chip
constexpr int LDS_WORKER_BYTES = 4 + 4 + 4 + 4 + 4 * PMAX + 4 * PMAX + 8 + 8 + 8 + 8 + 1;
constexpr int LDS_WORKERS_MAX = 1024;

// copy worker state between HBM (D.w_*) and the LDS carve (dir 0: load, 1: store back)
__device__ void workers_lds(const Dev& D, int dir) {
  const int W = D.W;
  int32_t* nth = (int32_t*)lds_field(W, 0);
  int32_t* cap = (int32_t*)lds_field(W, 1);
  int32_t* npr = (int32_t*)lds_field(W, 2);
  int32_t* pl = (int32_t*)lds_field(W, 3);
  int32_t* pf = (int32_t*)lds_field(W, 4);
  int32_t* pc = (int32_t*)lds_field(W, 5);
  int64_t* no = (int64_t*)lds_field(W, 6);
  int64_t* nb = (int64_t*)lds_field(W, 7);
  int64_t* its = (int64_t*)lds_field(W, 8);
  unsigned long long* lc = (unsigned long long*)lds_field(W, 9);
  uint8_t* fl = (uint8_t*)lds_field(W, 10);
  for (int w = threadIdx.x; w < W; w += blockDim.x) {
    if (dir == 0) {
      nth[w] = D.w_nthreads[w];
      cap[w] = D.w_cap[w];
      npr[w] = D.w_nproc[w];
      pl[w] = D.w_plen[w];
      no[w] = D.w_netocc[w];
      nb[w] = D.w_nbytes[w];
      its[w] = D.w_itcslots[w];
      lc[w] = D.w_lastcheck[w];
      fl[w] = D.w_flags[w];
    } else {
      D.w_nproc[w] = npr[w];
      D.w_plen[w] = pl[w];
      D.w_netocc[w] = no[w];
      D.w_nbytes[w] = nb[w];
      D.w_itcslots[w] = its[w];
      D.w_lastcheck[w] = lc[w];
      D.w_flags[w] = fl[w];
    }
  }
  for (int i = threadIdx.x; i < W * PMAX; i += blockDim.x) {
    if (dir == 0) {
      pf[i] = D.w_pfx[i];
      pc[i] = D.w_pcnt[i];
    } else {
      D.w_pfx[i] = pf[i];
      D.w_pcnt[i] = pc[i];
    }
  }
}

// the ordered commit of one round (one workgroup; owner[] and, for W <= 1024, the
// worker state in dynamic LDS)
__device__ void commit_body(const Dev& D, bool manage_lds) {
  int* owner = (int*)dgp_smem;
  __shared__ CoopShared S;
  __shared__ int s_base, s_gfirst, s_uniform, s_firstq, s_qbad, s_pop_prefix, s_resolved, s_err, s_isg, s_ncommit;
  __shared__ int s_commit[CTA];
  __shared__ int64_t s_stage_next;
  Ctl* c = D.ctl;
  const int n = (int)c->round_n;
  if (n == 0) return;
  unsigned long long t_0 = __builtin_amdgcn_s_memtime(), t_a;
  if (manage_lds && D.lds_workers) {
    workers_lds(D, 0);
    __syncthreads();
  }
  const int32_t* L = c->round_L;
  const unsigned long long tag = (unsigned long long)c->round_counter << 32;
  const int P = D.P;
  const int tid = threadIdx.x;

  // ---- durations in effect at each stimulus (TaskPrefix.add_duration EWMA, in order)
  if (tid == 0) {
    s_uniform = 1;
    s_firstq = INT32_MAX;
    s_qbad = 0;
    s_resolved = 0;
    s_err = 0;
  }
  __syncthreads();
  for (int j = tid; j < n; j += blockDim.x) {
    int t = L[j];
    double cur = D.pdur_cur[D.prefix[t]];
    if (!(cur >= 0 && D.res_stop[t] - D.res_start[t] == cur)) s_uniform = 0;
    if (D.ev_flags[j] & EV_MAYQUEUE) atomicMin(&s_firstq, j);
    D.ev_npl[j] = -1;  // not committed yet
  }
  __syncthreads();
  const bool uniform = s_uniform != 0;
  if (uniform) {
    for (int p = tid; p < P; p += blockDim.x) D.durv[p] = D.pdur_cur[p];
  } else {
    // one lane per prefix walks the stimuli in order
    for (int p = tid; p < P; p += blockDim.x) {
      double v = D.pdur_cur[p];
      for (int j = 0; j < n; j++) {
        int t = L[j];
        if (D.prefix[t] == p) v = ewma(v, D.res_stop[t] - D.res_start[t]);
        D.durv[(size_t)j * P + p] = v;
      }
      D.pdur_cur[p] = v;
    }
  }
  // ---- classification, queue bound, staging / record offsets
  const long long qlen0 = c->qlen;
  int64_t run_pop = 0, run_pub = 0, run_rub = 0;
  const int64_t rec0 = (int64_t)c->rec_used;
  if (qlen0 > 0 && tid == 0) s_pop_prefix = D.prefix[D.qarr[c->qhead]];
  __syncthreads();
  for (int j0 = 0; j0 < n; j0 += blockDim.x) {
    int j = j0 + tid;
    bool in = j < n;
    int popmax = (in && qlen0 > 0) ? D.w_cap[D.ev_w[j]] : 0;
    int64_t tot;
    int64_t pexcl = block_excl_scan(popmax, &tot);
    uint8_t fl = in ? D.ev_flags[j] : 0;
    if (in && popmax > 0 && run_pop + pexcl + popmax > qlen0) fl |= EV_GLOBAL;
    if (in && popmax > 56) fl |= EV_GLOBAL;  // records / placements of a local stimulus fit in one wave
    if (in && j > s_firstq) fl |= EV_GLOBAL;
    run_pop += tot;
    if (in) D.ev_flags[j] = fl;
    bool glob = (fl & EV_GLOBAL) != 0;
    int64_t pub = (in && !glob) ? D.ev_nf[j] + popmax : 0;
    int64_t rub = (in && !glob) ? 1 + D.ev_nf[j] + popmax : 0;
    if (in) D.ev_popmax[j] = glob ? 0 : popmax;
    int64_t po = block_excl_scan(pub, &tot);
    if (in) D.ev_plbase[j] = run_pub + po;
    run_pub += tot;
    int64_t ro = block_excl_scan(rub, &tot);
    if (in) D.ev_recbase[j] = rec0 + run_rub + ro;
    run_rub += tot;
  }
  if (qlen0 > 0) {
    int64_t rng = run_pop < qlen0 ? run_pop : qlen0;
    for (int64_t i = tid; i < rng; i += blockDim.x) {
      int q = D.qarr[c->qhead + i];
      if (D.dep_ptr[q + 1] != D.dep_ptr[q] || D.prefix[q] != s_pop_prefix) s_qbad = 1;
    }
    __syncthreads();
    if (s_qbad)
      for (int j = tid; j < n; j += blockDim.x)
        if (D.ev_popmax[j] > 0) {
          D.ev_flags[j] |= EV_GLOBAL;
          D.ev_popmax[j] = 0;  // its reserved slots stay unused (REC_NONE / not copied)
        }
  }
  if (rec0 + run_rub > D.rec_cap || run_pub > D.st_cap) {
    if (tid == 0) set_error(D, rec0 + run_rub > D.rec_cap ? ERR_REC_CAP : ERR_STAGE_CAP, -1);
    if (manage_lds && D.lds_workers) {
      __syncthreads();
      workers_lds(D, 1);
    }
    return;
  }
  for (int64_t i = tid; i < run_rub; i += blockDim.x) D.rec[rec0 + i].kind = REC_NONE;
  for (int i = tid; i < D.W; i += blockDim.x) owner[i] = INT32_MAX;
  if (tid == 0) {
    c->rec_used = (unsigned long long)(rec0 + run_rub);
    s_stage_next = run_pub;
    s_base = 0;
  }
  __threadfence_block();
  __syncthreads();
  t_a = __builtin_amdgcn_s_memtime();
  if (tid == 0) c->prof[0] += t_a - t_0;

  // ---- deterministic-reservation commit over the slice [base, base + CTA)
  while (true) {
    unsigned long long ts0 = __builtin_amdgcn_s_memtime();
    const int base = s_base;
    if (base >= n || s_err) break;
    if (tid == 0) {
      s_isg = (D.ev_flags[base] & EV_GLOBAL) ? 1 : 0;
      s_gfirst = INT32_MAX;
      s_ncommit = 0;
    }
    __syncthreads();
    if (s_isg) {
      const double* dur = D.durv + (uniform ? 0 : (size_t)base * P);
      int64_t sn = s_stage_next;
      int resolved = s_resolved;
      exec_global(D, L, base, tag | (unsigned long long)base, dur, S, &sn, &resolved);
      if (tid == 0) {
        s_stage_next = sn;
        s_resolved = resolved;
        if (sn > D.st_cap) set_error(D, ERR_STAGE_CAP, -1);
        int b = base + 1;
        while (b < n && D.ev_npl[b] >= 0) b++;
        s_base = b;
        s_err = c->error;
        c->prof[2] += __builtin_amdgcn_s_memtime() - ts0;
      }
      __syncthreads();
      continue;
    }
    const int j = base + tid;
    const bool pending = j < n && D.ev_npl[j] < 0;
    if (pending && (D.ev_flags[j] & EV_GLOBAL)) atomicMin(&s_gfirst, j);
    __syncthreads();
    const bool active = pending && j < s_gfirst;
    const int32_t* touch = D.ev_touch + (size_t)(active ? j : 0) * TOUCH_MAX;
    const int nt = active ? D.ev_ntouch[j] : 0;
    for (int i = 0; i < nt; i++) atomicMin(&owner[touch[i]], j);
    __syncthreads();
    bool mine = active;
    for (int i = 0; i < nt && mine; i++) mine = owner[touch[i]] == j;
    unsigned long long ts1 = __builtin_amdgcn_s_memtime();
    if (mine) s_commit[atomicAdd(&s_ncommit, 1)] = j;
    __syncthreads();
    {
      const int nc = s_ncommit;
      for (int q = tid >> 6; q < nc; q += blockDim.x >> 6) {
        const int jj = s_commit[q];
        const double* dur = D.durv + (uniform ? 0 : (size_t)jj * P);
        const unsigned long long kk = tag | (unsigned long long)jj;
        unsigned long long tx = __builtin_amdgcn_s_memtime();
        if (D.lds_workers)
          exec_local_wave<true>(D, jj, L[jj], D.ev_w[jj], kk, dur, D.ev_plbase[jj], D.ev_recbase[jj],
                                D.ev_popmax[jj], qlen0 > 0 ? s_pop_prefix : 0);
        else
          exec_local_wave<false>(D, jj, L[jj], D.ev_w[jj], kk, dur, D.ev_plbase[jj], D.ev_recbase[jj],
                                 D.ev_popmax[jj], qlen0 > 0 ? s_pop_prefix : 0);
        if ((tid & 63) == 0) {
          unsigned long long dx = __builtin_amdgcn_s_memtime() - tx;
          atomicMax(&c->prof[6], dx);
          atomicAdd(&c->prof[7], dx);
        }
      }
    }
    __syncthreads();
    if (tid == 0) c->prof[4] += ts1 - ts0;  // reservation part of the step
    for (int i = 0; i < nt; i++) owner[touch[i]] = INT32_MAX;
    if (tid == 0) {
      int b = base;
      while (b < n && D.ev_npl[b] >= 0) b++;
      s_base = b;
      c->dr_steps++;
      s_err = c->error;
      unsigned long long dt = __builtin_amdgcn_s_memtime() - ts0;
      c->prof[1] += dt;
      if (dt > c->prof[5]) c->prof[5] = dt;
    }
    __syncthreads();
  }
  __syncthreads();
  unsigned long long t_f = __builtin_amdgcn_s_memtime();
  // ---- queued tasks taken by local stimuli, then the placement log in stimulus order
  resolve_pops_coop(D, L, s_resolved, n);
  int64_t run = 0;
  const int64_t dst0 = (int64_t)c->n_placed;
  for (int j0 = 0; j0 < n; j0 += blockDim.x) {
    int j = j0 + tid;
    int64_t cnt = j < n ? D.ev_npl[j] : 0;
    if (cnt < 0) cnt = 0;
    int64_t tot;
    int64_t off = block_excl_scan(cnt, &tot);
    if (cnt > 0) {
      int64_t src = D.ev_plbase[j], dst = dst0 + run + off;
      for (int64_t i = 0; i < cnt; i++) {
        D.pl_task[dst + i] = D.st_task[src + i];
        D.pl_worker[dst + i] = D.st_worker[src + i];
        D.pl_comm[dst + i] = D.st_comm[src + i];
        D.pl_start[dst + i] = D.st_start[src + i];
        D.pl_wsnbytes[dst + i] = D.st_wsnbytes[src + i];
        D.pl_route[dst + i] = D.st_route[src + i];
      }
    }
    run += tot;
  }
  __syncthreads();
  if (tid == 0) c->n_placed = (unsigned long long)(dst0 + run);
  if (manage_lds && D.lds_workers) {
    __syncthreads();
    workers_lds(D, 1);
  }
  if (tid == 0) c->prof[3] += __builtin_amdgcn_s_memtime() - t_f;
}
__global__ void __launch_bounds__(CTA) k_commit(const Dev* __restrict__ Dp) { commit_body(*Dp, true); }

// fold the whole record log into idle / saturated (single lane)
__global__ void k_walk(const Dev* __restrict__ Dp) {
  const Dev& D = *Dp;
  if (threadIdx.x == 0 && blockIdx.x == 0) walk_to(D, D.ctl->rec_used);
}

__device__ void snapshot_body(const Dev& D, long long* prev_placed, int after_round, int64_t gtid, int64_t gthreads,
                              bool leader) {
  if (after_round && D.ctl->round_n == 0) return;
  int64_t r = D.ctl->rounds_nonempty;
  if (r >= D.snap_cap) return;
  for (int64_t w = gtid; w < D.W; w += gthreads) {
    size_t o = (size_t)r * D.W + w;
    D.snap_occ[o] = occupancy(D, w, D.pdur_cur);
    D.snap_nbytes[o] = WK_nbytes(D)[w];
    D.snap_nproc[o] = WK_nproc(D)[w];
    D.snap_flags[o] = WK_flags(D)[w];
  }
  if (leader) {
    D.snap_nplaced[r] = (int32_t)((long long)D.ctl->n_placed - *prev_placed);
    D.snap_nqueued[r] = (int32_t)D.ctl->qlen;
    *prev_placed = (long long)D.ctl->n_placed;
  }
}
__global__ void k_snapshot(const Dev* __restrict__ Dp, long long* prev_placed, int after_round) {
  snapshot_body(*Dp, prev_placed, after_round, blockIdx.x * (int64_t)blockDim.x + threadIdx.x,
                (int64_t)gridDim.x * blockDim.x, blockIdx.x == 0 && threadIdx.x == 0);
}

// the whole synthetic-executor replay in one workgroup: every phase of every round runs
// on the commit's CU, so the round's data stays in its L1 / L2 and worker state stays in
// LDS for the whole replay; no launches or host synchronisation between rounds
__global__ void __launch_bounds__(CTA) k_replay(const Dev* __restrict__ Dp, long long* next_start, long long max_rounds,
                                                long long* prev_placed, int snapshots) {
  const Dev& D = *Dp;
  __shared__ long long s_n;
  __shared__ int s_stop;
  if (D.lds_workers) workers_lds(D, 0);
  __syncthreads();
  for (long long r = 0; max_rounds < 0 || r < max_rounds; r++) {
    if (threadIdx.x == 0) {
      round_begin(D, next_start, nullptr, 0);
      s_n = D.ctl->round_n;
      s_stop = D.ctl->error != 0;
    }
    __threadfence_block();
    __syncthreads();
    if (s_n == 0 || s_stop) break;
    frontier_release_body(D, threadIdx.x, blockDim.x);
    __threadfence_block();
    __syncthreads();
    candidate_body(D, threadIdx.x >> 6, blockDim.x >> 6);
    __threadfence_block();
    __syncthreads();
    events_body(D, threadIdx.x, blockDim.x);
    __threadfence_block();
    __syncthreads();
    commit_body(D, false);
    __threadfence_block();
    __syncthreads();
    if (snapshots) {
      if (threadIdx.x == 0) walk_to(D, D.ctl->rec_used);
      __threadfence_block();
      __syncthreads();
      snapshot_body(D, prev_placed, 1, threadIdx.x, blockDim.x, threadIdx.x == 0);
      __threadfence_block();
      __syncthreads();
    }
  }
  __syncthreads();
  if (D.lds_workers) workers_lds(D, 1);
}

}  // namespace dgp
