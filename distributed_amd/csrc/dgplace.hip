// dgplace — MI355X (gfx950) placement engine for the dask.distributed scheduler hot path.
//
// Host side of the C ABI declared in include/dgplace.h; the device side (state layout,
// kernels, the deterministic-reservation commit) is in dgp_device.h.
//
// Device-resident state (HBM): the task graph as CSR dependencies + dependents (rows in
// ascending priority), per-task replica bitsets who_has[N][ceil(W/64)], task states and
// counters, per-worker occupancy state, the placement log and the record log.
// A replay = k_ug_init + k_ug_dispatch (the update_graph stimulus), then rounds of
// k_round_begin, k_frontier_release, k_candidate_commbytes, k_events, k_commit enqueued
// back to back without host synchronisation (the device decides when a round is empty),
// then k_walk (idle / saturated sets up to date).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/dgplace.h"
#include "dgp_device.h"
#include "dgp_msgs.h"
#include "dgp_stream.h"  // dgp::st: the 32-slot window with wait-in-place claims
#undef DGP_ST_NS
#undef DGP_WIN
#undef DGP_WAITC
#define DGP_ST_NS st64  // dgp::st64: the same stream kernel with 64 slots, no wait-in-place
#define DGP_WIN 64
#define DGP_WAITC 0
#include "dgp_stream.h"
#include "dgp_events.h"
#include "dgp_steal.h"
#include "dgp_service.h"

#include <hipcub/hipcub.hpp>

// =================================================================== host side

struct StealCtx {  // WorkStealing arrays of the last dgp_steal_load (one arena)
  char* arena = nullptr;
  size_t cap = 0;
  dgp::steal::Prob P{};
  void* d_tmp = nullptr;
  size_t tmp_bytes = 0;
  int32_t* keys_sorted = nullptr;
  int32_t* d_vals = nullptr;
  int32_t W = 0;
  int64_t T = 0;
  int NK = 0;
  int64_t n_stealable = 0;
  bool loaded = false;
  // dgp_steal_order for the next load: the tasks' (priority, arrival) keys (host)
  std::vector<int64_t> order_prio, order_arr;
};

struct dgp_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  dgp::Dev D{};
  int window = 32;  // the stream kernel build the next launch runs (dgp_set_window): 32 or 64
  // what the device copies of D hold (d_dev, the stream kernel's c_dev symbol) and the
  // dynamic-LDS size last set on each stream kernel: unchanged ones are not re-sent
  dgp::Dev dev_sent[2]{};
  bool dev_valid = false;
  dgp::Ctl* ctl = nullptr;
  long long* d_aux = nullptr;  // [0] next round start, [1] placements at the last snapshot,
                               // [2] service stimuli consumed by the round engine,
                               // [3] messages one k_svc_append call answered
  dgp::Dev* d_dev = nullptr;    // [0] Dev for every kernel, [1] Dev with lds_workers for k_commit
  std::vector<void*> allocs;
  std::vector<void*> graph_allocs;
  bool have_config = false, have_workers = false, have_graph = false, have_results = false;
  bool graph_done = false;
  int64_t snap_rounds = 0;
  std::vector<int32_t> nthreads;
  std::vector<double> prefix_defaults;
  std::vector<int64_t> group_sizes;
  int64_t E = 0;
  int rounds_per_sync = 16;
  bool stream_used = false;  // the stream engine ran: the round-kernel path is no longer valid
  int mode = 0;              // 0 fresh, 1 replay (dgp_run_rounds), 2 service (dgp_tasks_finished)
  dgp::svc::Msg* d_msgs = nullptr;  // service-mode message batch (device) + status
  int8_t* d_status = nullptr;
  dgp::svc::Msg* h_msgs = nullptr;  // pinned staging of the batch
  int64_t msgs_cap = 0;
  unsigned long long last_placed = 0;  // placement-log length after the last synchronising call
  // timing: (start, stop) event pairs recorded around launches, resolved lazily
  bool timing = false;
  double kms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t klaunch[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  std::vector<hipEvent_t> evpool;
  std::vector<int> evkind;
  size_t evused = 0;
  StealCtx steal;
  std::vector<uint8_t> tflags_h;           // task flags as set_graph computed them
  std::vector<int32_t> group_h;            // TaskGroup of each task
  std::vector<int64_t> h_dep_ptr, h_prio;  // the uploaded graph (dgp_add_graph appends to it)
  std::vector<int32_t> h_wide;             // tasks with more than UG_WIDE dependencies (k_ug_init_wide)
  int64_t* d_rdy = nullptr;                // update_graph's ready-list pass: per-tile counts, then the total
  int64_t rdy_cap = 0;
  std::vector<int32_t> h_dep_idx, h_prefix;
  std::vector<uint8_t> h_wanted;
  std::vector<int64_t> gdep_n, gdep_len;   // per group: len(tg.dependencies), sum of their lengths
  std::vector<int8_t> rootish_override_h;  // TaskState._rootish per task (-1: None)
  std::vector<uint8_t> restr_h;            // restriction flags per task (empty: none)
  int64_t rpool_used = 0, rpool_cap = 0;    // dgp_update_restrictions' row pool on the device (int32s)
  std::vector<uint8_t> paused_h;           // per worker: 0 running, 1 paused, 2 removed
  int64_t log_min[3] = {0, 0, 0};          // minimum capacities of the placement / stimulus / record logs
  int64_t sv_used = 0;                     // service stimuli appended (accepted task-finished messages)
  char* d_ev = nullptr;                    // service-event argument staging (device)
  size_t d_ev_cap = 0;
  char* d_msgbuf = nullptr;                // dgp_task_messages scratch (device)
  size_t d_msgbuf_cap = 0;
  // resident service mode (dgp_set_resident): the stream kernel stays launched between
  // dgp_tasks_finished calls and takes each batch from a mailbox in pinned host memory
  dgp::svc::Mbox* mb = nullptr;      // host address
  dgp::svc::Mbox* mb_dev = nullptr;  // device address
  bool resident = false;             // service calls go through the resident kernel
  bool res_msgs = false;             // the resident answers carry the compute-task message fields
  bool res_running = false;          // the resident kernel was launched (it may have ended since)
  bool res_hung = false;             // the resident kernel did not end when told to: the engine is unusable
  bool pending_resync = false;       // a later graph with dependencies on earlier tasks: dgp_sync_* next
  int64_t pending_lo = -1;           // ... its first task (dgp_graph_stimulus may run its stimulus instead)
  unsigned long long req_seq = 0;    // the last request number sent
  // dgp_tasks_finished_post: 0 nothing posted, 1 a batch in the resident mailbox awaiting its
  // answer, 2 answered at the post (launch per call) and kept for dgp_tasks_finished_wait
  int posted = 0;
  int64_t posted_n = 0, posted_new = 0;
  std::vector<int8_t> posted_status;
  int64_t res_prof[4] = {0, 0, 0, 0};  // requests answered; sums of append, run, publish (device 100 MHz ticks)
  int64_t res_role[7] = {0, 0, 0, 0, 0, 0, 0};  // sums of each role's last batch end after the append
};

namespace {

int fail(dgp_engine* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  return code;
}

#define HIPCHK(e, call)                                                              \
  do {                                                                               \
    hipError_t _st = (call);                                                         \
    if (_st != hipSuccess)                                                           \
      return fail(e, DGP_E_HIP, std::string(#call) + ": " + hipGetErrorString(_st)); \
  } while (0)

template <class T>
int dalloc(dgp_engine* e, T** p, size_t count, std::vector<void*>& list) {
  if (count == 0) count = 1;
  hipError_t st = hipMalloc((void**)p, count * sizeof(T));
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(st));
  list.push_back((void*)*p);
  return 0;
}

// grow a device array from n0 to n1 elements: the first n0 copied, the rest zero; the
// allocation list entry follows the new pointer
template <class T>
int regrow(dgp_engine* e, T** p, size_t n0, size_t n1, std::vector<void*>& list) {
  T* q = nullptr;
  hipError_t st = hipMalloc((void**)&q, std::max<size_t>(n1, 1) * sizeof(T));
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(st));
  HIPCHK(e, hipMemsetAsync(q, 0, std::max<size_t>(n1, 1) * sizeof(T), e->stream));
  if (*p && n0) HIPCHK(e, hipMemcpyAsync(q, *p, std::min(n0, n1) * sizeof(T), hipMemcpyDeviceToDevice, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  bool found = false;
  for (auto& x : list)
    if (x == (void*)*p) {
      x = (void*)q;
      found = true;
    }
  if (*p && found) (void)hipFree(*p);
  if (!found) list.push_back((void*)q);
  *p = q;
  return 0;
}
// re-stride a [rows][w0] device array to [rows][w1] (w1 >= w0): each row copied, the new
// columns zero
template <class T>
int restride(dgp_engine* e, T** p, size_t rows, size_t w0, size_t w1, std::vector<void*>& list) {
  T* q = nullptr;
  hipError_t st = hipMalloc((void**)&q, std::max<size_t>(rows * w1, 1) * sizeof(T));
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(st));
  HIPCHK(e, hipMemsetAsync(q, 0, std::max<size_t>(rows * w1, 1) * sizeof(T), e->stream));
  if (*p && rows && w0)
    HIPCHK(e, hipMemcpy2DAsync(q, w1 * sizeof(T), *p, w0 * sizeof(T), w0 * sizeof(T), rows, hipMemcpyDeviceToDevice,
                               e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  bool found = false;
  for (auto& x : list)
    if (x == (void*)*p) {
      x = (void*)q;
      found = true;
    }
  if (*p && found) (void)hipFree(*p);
  if (!found) list.push_back((void*)q);
  *p = q;
  return 0;
}

// open row `pos` of a [W0 + 1][row] device array whose rows 0..W0-1 are in use: rows
// pos..W0-1 move up by one, row pos zero (a worker inserted at index pos)
template <class T>
int shift_rows(dgp_engine* e, T* p, size_t W0, size_t row, size_t pos) {
  if (!p || pos >= W0) return 0;
  std::vector<T> h((W0 + 1) * row);
  HIPCHK(e, hipMemcpy(h.data(), p, h.size() * sizeof(T), hipMemcpyDeviceToHost));
  std::memmove(h.data() + (pos + 1) * row, h.data() + pos * row, (W0 - pos) * row * sizeof(T));
  std::fill(h.data() + pos * row, h.data() + (pos + 1) * row, T{});
  HIPCHK(e, hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

void free_list(std::vector<void*>& l) {
  for (void* p : l) (void)hipFree(p);
  l.clear();
}

int read_ctl(dgp_engine* e, dgp::Ctl* c) {
  HIPCHK(e, hipMemcpyAsync(c, e->ctl, sizeof *c, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return 0;
}

int check_device_error(dgp_engine* e, dgp::Ctl* out = nullptr) {
  dgp::Ctl c;
  if (int rc = read_ctl(e, &c)) return rc;
  if (out) *out = c;
  if (c.error) {
    static const char* names[] = {"none", "worker prefix dict overflow (PMAX)", "task without candidates",
                                  "inconsistent task state", "queue underflow", "candidate pool overflow",
                                  "global prefix dict overflow", "record log overflow", "staging overflow",
                                  "no worker", "needs_what line overflow", "prefix dict overflow (stream)",
                                  "watchdog: the stream engine made no progress", "queue", "needs_what inconsistent",
                                  "record log overflow (stream)", "task without candidates (stream)",
                                  "descriptor ring out of order", "worker index out of range (stream)", "stream invariant violated",
                                  "a service event the engine does not model"};
    char buf[200];
    snprintf(buf, sizeof buf, "device engine error %d (%s) at task %d", c.error,
             (c.error >= 0 && c.error <= 20) ? names[c.error] : "?", c.err_task);
    if (c.error == dgp::ERR_UNSUPPORTED) {  // a refused event changed nothing: the engine stays usable
      const int zero[2] = {0, -1};
      HIPCHK(e, hipMemcpy((char*)e->ctl + offsetof(dgp::Ctl, error), zero, sizeof zero, hipMemcpyHostToDevice));
    }
    return fail(e, DGP_E_DEVICE, buf);
  }
  return 0;
}

// End the resident service kernel (it writes the engine state back as any launch does).
// Every entry point but dgp_tasks_finished calls this first: nothing else may touch the
// engine's stream or device state while it runs.
int resident_stop(dgp_engine* e) {
  if (e && e->res_hung) return fail(e, DGP_E_DEVICE, "the resident kernel did not end: the engine is unusable");
  if (e && e->posted) return fail(e, DGP_E_STATE, "a posted task-finished batch: dgp_tasks_finished_wait first");
  if (!e || !e->res_running) return 0;
  __atomic_store_n(&e->mb->stop, 1, __ATOMIC_RELEASE);
  const hipError_t st = hipStreamSynchronize(e->stream);
  __atomic_store_n(&e->mb->stop, 0, __ATOMIC_RELEASE);
  e->res_running = false;
  e->D.resident = 0;
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("resident kernel: ") + hipGetErrorString(st));
  return 0;
}

int resident_wait(dgp_engine* e, int8_t* status, int64_t* n_new_placements);  // below

// A kernel's static LDS bytes as built (the module-wide LDS lowering, build.py, allocates
// every LDS variable its out-of-line callees use at fixed addresses in the kernel's block)
size_t kernel_static_lds(const void* fn, size_t fallback) {
  hipFuncAttributes a;
  if (hipFuncGetAttributes(&a, fn) != hipSuccess) return fallback > 32 * 1024 ? fallback : 32 * 1024;
  return a.sharedSizeBytes;
}

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

// publish the host-side Dev (pointers, sizes, config) to the device copies the kernels read
int sync_dev(dgp_engine* e) {
  const char* dbg = getenv("DGP_STREAM_DEBUG");
  e->D.dbg = dbg ? atoi(dbg) : 0;
  const char* dt = getenv("DGP_DEBUG_TASK");
  e->D.dbg_task = dt ? atoi(dt) : -2;
  const char* pl = getenv("DGP_PRE_LEAD");
  e->D.pre_lead = pl ? atoi(pl) : dgp::st::DR;
  if (e->D.pre_lead < 64 || e->D.pre_lead > dgp::st::DR) e->D.pre_lead = dgp::st::DR;
  if (!e->D.dbgbuf) HIPCHK(e, hipMalloc((void**)&e->D.dbgbuf, 64 * 8 * sizeof(double)));
  if (const char* tl = getenv("DGP_TRACE_LO")) {  // DGP_TRACE builds: sampled lifecycle trace
    const char* tn = getenv("DGP_TRACE_N");
    e->D.trace_lo = atoll(tl);
    const long long n = tn ? atoll(tn) : 20000;
    if (!e->D.trace || e->D.trace_n != n) {
      if (e->D.trace) (void)hipFree(e->D.trace);
      HIPCHK(e, hipMalloc((void**)&e->D.trace, n * 32 * 8));
    }
    e->D.trace_n = n;
    HIPCHK(e, hipMemset(e->D.trace, 0, n * 32 * 8));
  }
  // the stream engine owns the worker state (and its needs_what layout) whenever it runs
  e->D.needs_stream = e->D.gw_needs_saved && e->D.P <= dgp::st::PX ? 1 : 0;
  dgp::Dev h[2] = {e->D, e->D};
  h[0].lds_workers = 0;
  h[1].lds_workers = e->D.W <= dgp::LDS_WORKERS_MAX ? 1 : 0;
  if (e->dev_valid && !memcmp(h, e->dev_sent, sizeof h)) return 0;  // the device copy is current
  HIPCHK(e, hipMemcpy(e->d_dev, h, sizeof h, hipMemcpyHostToDevice));
  memcpy(e->dev_sent, h, sizeof h);
  e->dev_valid = true;
  return 0;
}

int grid_for(int64_t n, int per_block, int cap) {
  int64_t b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

// run_id / holder_of of the placements the stream engine has not sequenced itself
int set_runids(dgp_engine* e) {
  hipLaunchKernelGGL(dgp::svc::k_set_runids, dim3(64), dim3(256), 0, e->stream, e->d_dev);
  hipLaunchKernelGGL(dgp::svc::k_set_runids_done, dim3(1), dim3(64), 0, e->stream, e->d_dev);
  HIPCHK(e, hipGetLastError());
  return 0;
}

// Service sessions can place and complete a task more than once (rescheduled, recomputed
// after a worker loss): before a call that may place up to every task and append up to
// `stimuli` completions, the logs grow (doubling) so that one call cannot overflow them.
int grow_logs(dgp_engine* e, int64_t stimuli) {
  dgp::Dev& D = e->D;
  const int64_t N = D.N, used_pl = (int64_t)e->last_placed;
  auto& L = e->graph_allocs;
  int rc = 0;
  if (used_pl + N + 64 > D.pl_cap) {
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const int64_t cap = std::max<int64_t>(2 * D.pl_cap, used_pl + N + 64);
    rc |= regrow(e, &D.pl_task, D.pl_cap, cap, L);
    rc |= regrow(e, &D.pl_worker, D.pl_cap, cap, L);
    rc |= regrow(e, &D.pl_comm, D.pl_cap, cap, L);
    rc |= regrow(e, &D.pl_start, D.pl_cap, cap, L);
    rc |= regrow(e, &D.pl_wsnbytes, D.pl_cap, cap, L);
    rc |= regrow(e, &D.pl_route, D.pl_cap, cap, L);
    if (rc) return rc;
    D.pl_cap = cap;
  }
  if (e->sv_used + stimuli > D.sv_cap) {
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const int64_t cap = std::max<int64_t>(2 * D.sv_cap, e->sv_used + stimuli);
    rc |= regrow(e, &D.sv_task, D.sv_cap, cap, L);
    rc |= regrow(e, &D.sv_worker, D.sv_cap, cap, L);
    if (rc) return rc;
    D.sv_cap = cap;
  }
  // one record per placement and per completion
  if (used_pl + N + e->sv_used + stimuli + 4096 > D.rlog_cap) {
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const int64_t cap = std::max<int64_t>(2 * D.rlog_cap, used_pl + N + e->sv_used + stimuli + 4096);
    rc |= regrow(e, &D.rlog, D.rlog_cap, cap, L);
    if (rc) return rc;
    D.rlog_cap = cap;
  }
  return 0;
}

// the stimulus source of the stream engine for the coming launch
// k_ug_dispatch: which of its arrays go to dynamic LDS (in the order below, while they fit
// beside the kernel's static LDS), and that many bytes
void ug_lds_plan(const dgp::Dev& D, uint32_t* mask, size_t* bytes) {
  static size_t stat = 0;
  if (!stat) stat = kernel_static_lds((const void*)dgp::k_ug_dispatch, 48 * 1024);
  const size_t budget = 160 * 1024 > stat + 1024 ? 160 * 1024 - stat - 1024 : 0;
  uint32_t m = 0;
  size_t used = 0;
  // the prefix durations first (a few hundred bytes, read by every occupancy), then the
  // list in order while it fits
  const int order[dgp::UG_NF] = {13, 14, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12};
  for (int k : order) {
    const size_t b = (dgp::ug_field_bytes(k, D.W, D.Wp, D.P) + 15) & ~(size_t)15;
    if (used + b > budget) break;
    used += b;
    m |= 1u << k;
  }
  *mask = m;
  *bytes = used;
}

// update_graph part 1 over tasks [lo, N): k_ug_init, then k_ug_init_wide for each row wider
// than UG_WIDE (counted across a grid instead of one wave's serial loop)
int launch_ug_init(dgp_engine* e, int64_t lo) {
  const dgp::Dev* DP = e->d_dev;
  hipStream_t s = e->stream;
  const int64_t N = e->D.N;
  hipLaunchKernelGGL(dgp::k_ug_init, dim3(grid_for(N - lo, 256, 2048)), dim3(256), 0, s, DP, (int)lo);
  for (int32_t t : e->h_wide) {
    if (t < lo) continue;
    const int64_t a = e->h_dep_ptr[t], b = e->h_dep_ptr[t + 1];
    hipLaunchKernelGGL(dgp::k_ug_init_wide, dim3(grid_for(b - a, 1024, 256)), dim3(256), 0, s, DP, (int)t, a, b);
  }
  return 0;
}

int launch_ug_dispatch(dgp_engine* e, int scan_lo, int task_lo) {
  uint32_t mask = 0;
  size_t bytes = 0;
  ug_lds_plan(e->D, &mask, &bytes);
  static size_t attr_set[64];
  if (bytes > attr_set[e->device & 63]) {
    HIPCHK(e, hipFuncSetAttribute((const void*)dgp::k_ug_dispatch, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    attr_set[e->device & 63] = bytes;
  }
  // the ready list's tiles: a count per tile, then the total
  const int64_t n_scan = std::max<int64_t>(0, (int64_t)e->D.N - scan_lo);
  const int64_t tiles = (n_scan + dgp::RDY_TILE - 1) / dgp::RDY_TILE;
  if (tiles + 1 > e->rdy_cap) {
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->d_rdy) HIPCHK(e, hipFree(e->d_rdy));
    e->d_rdy = nullptr;
    e->rdy_cap = 0;
    const int64_t cap = std::max<int64_t>(tiles + 1, 1024);
    HIPCHK(e, hipMalloc((void**)&e->d_rdy, (size_t)cap * 8));
    e->rdy_cap = cap;
  }
  int64_t* total = e->d_rdy + tiles;
  const dgp::Dev* DP = e->d_dev;
  hipStream_t s = e->stream;
  return timed_launch(e, 3, [&] {
    if (tiles == 0) {
      (void)hipMemsetAsync(total, 0, 8, s);
    } else {
      hipLaunchKernelGGL(dgp::k_ready_count, dim3((unsigned)tiles), dim3(dgp::CTA), 0, s, DP, scan_lo, task_lo, e->d_rdy);
      hipLaunchKernelGGL(dgp::k_ready_scatter, dim3((unsigned)tiles), dim3(dgp::CTA), 0, s, DP, scan_lo, task_lo,
                         (const int64_t*)e->d_rdy, total);
    }
    hipLaunchKernelGGL(dgp::k_ug_dispatch, dim3(1), dim3(dgp::CTA), bytes, s, DP, (const int64_t*)total, task_lo, mask);
  });
}

void stream_source(dgp_engine* e, bool service) {
  dgp::Dev& D = e->D;
  D.svc = service ? 1 : 0;
  D.stim_task = service ? D.sv_task : D.pl_task;
  D.stim_worker = service ? D.sv_worker : D.pl_worker;
  D.cseq = service ? D.sv_cseq : D.run_id;
}

// the two builds of the stream kernel (dgp_stream.h included as dgp::st and dgp::st64)
struct StreamW32 {
  static const void* kernel(bool lw) {
    return lw ? (const void*)dgp::st::k_stream<true> : (const void*)dgp::st::k_stream<false>;
  }
  static hipError_t send(const dgp::Dev& d, hipStream_t s) {
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(dgp::st::c_dev), &d, sizeof(dgp::Dev), 0, hipMemcpyHostToDevice, s);
  }
};
struct StreamW64 {
  static const void* kernel(bool lw) {
    return lw ? (const void*)dgp::st64::k_stream<true> : (const void*)dgp::st64::k_stream<false>;
  }
  static hipError_t send(const dgp::Dev& d, hipStream_t s) {
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(dgp::st64::c_dev), &d, sizeof(dgp::Dev), 0, hipMemcpyHostToDevice, s);
  }
};

// one launch of the stream kernel over the stimulus source set by stream_source()
template <class B>
int launch_stream_build(dgp_engine* e, long long max_rounds, int snaps) {
  const dgp::Dev& D = e->D;
  const size_t lds_w = dgp::st::lds_worker_bytes(D.W);
  // the kernel's static LDS (module-wide LDS lowering can place more than SLds in it)
  static size_t stat_lds = 0;
  if (!stat_lds) stat_lds = kernel_static_lds(B::kernel(true), dgp::ST_LDS_BYTES);
  const bool lw = stat_lds + lds_w <= 160 * 1024;
  // c_dev is one symbol per device and build, shared by every engine on it: re-sent unless it
  // holds exactly this engine's Dev already (content compare; engines are driven from one thread)
  static struct {
    bool valid;
    dgp::Dev v;
  } sent[64];
  auto& cs = sent[e->device & 63];
  if (!cs.valid || memcmp(&cs.v, &e->D, sizeof(dgp::Dev))) {
    HIPCHK(e, B::send(e->D, e->stream));
    cs.v = e->D;
    cs.valid = true;
  }
  long long mr = max_rounds;
  int sn = snaps;
  void* args[] = {&mr, &sn};
  const void* fn = B::kernel(lw);
  static size_t lds_max[64];  // the kernel attribute is per device: an upper bound, raised when needed
  if (lw && lds_max[e->device & 63] < lds_w) {
    HIPCHK(e, hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_w));
    lds_max[e->device & 63] = lds_w;
  }
  // ONE workgroup: every hand-off between the roles stays on this CU
  hipError_t lst = hipSuccess;
  if (int rc = timed_launch(e, 2, [&] {
        lst = hipLaunchKernel(fn, dim3(1), dim3(dgp::st::SCTA), args, lw ? lds_w : 0, e->stream);
      }))
    return rc;
  if (lst != hipSuccess) return fail(e, DGP_E_HIP, std::string("stream launch: ") + hipGetErrorString(lst));
  e->stream_used = true;
  return 0;
}

int launch_stream(dgp_engine* e, long long max_rounds, int snaps) {
  return e->window == 64 ? launch_stream_build<StreamW64>(e, max_rounds, snaps)
                         : launch_stream_build<StreamW32>(e, max_rounds, snaps);
}

int walk(dgp_engine* e) {
  const dgp::Dev* DP = e->d_dev;
  return timed_launch(e, 3, [&] { hipLaunchKernelGGL(dgp::k_walk, dim3(1), dim3(64), 0, e->stream, DP); });
}

// run the stimuli appended since the last launch: the stream engine, or one round of the
// round-kernel engine when the graph has more prefixes than the stream descriptors carry
// or worker restrictions
int run_service_stimuli(dgp_engine* e) {
  namespace V = dgp::svc;
  hipStream_t s = e->stream;
  if (e->D.P <= dgp::st::PX) {
    stream_source(e, true);
    if (int rc = launch_stream(e, -1, 0)) return rc;
  } else {
    // more prefixes than the stream descriptors carry, or restrictions: the accepted batch is one round of
    // the round-kernel engine (completions in message order)
    const dgp::Dev* DP = e->d_dev;
    const dgp::Dev* DPC = e->d_dev + 1;
    const int64_t N = e->D.N;
    const int big = grid_for(N, 256, 128);
    const int lds_workers = e->D.W <= dgp::LDS_WORKERS_MAX ? 1 : 0;
    const size_t lds = (((size_t)e->D.W * sizeof(int) + 15) & ~(size_t)15) +
                       (lds_workers ? (((size_t)e->D.W + 3) & ~(size_t)3) * dgp::LDS_WORKER_BYTES + 64 : 0);
    if (lds + kernel_static_lds((const void*)dgp::k_replay, 0) > 160 * 1024)
      return fail(e, DGP_E_ARG, "commit LDS exceeds 160 KiB");
    hipLaunchKernelGGL(V::k_svc_round_begin, dim3(1), dim3(64), 0, s, DP, e->d_aux + 2);
    if (int rc = timed_launch(e, 0, [&] { hipLaunchKernelGGL(dgp::k_frontier_release, dim3(big), dim3(256), 0, s, DP); }))
      return rc;
    if (int rc = timed_launch(e, 1, [&] {
          hipLaunchKernelGGL(dgp::k_candidate_commbytes, dim3(grid_for(N, 4, 256)), dim3(256), 0, s, DP);
        }))
      return rc;
    if (int rc = timed_launch(e, 3, [&] { hipLaunchKernelGGL(dgp::k_events, dim3(big), dim3(256), 0, s, DP); }))
      return rc;
    if (int rc = timed_launch(e, 2, [&] { hipLaunchKernelGGL(dgp::k_commit, dim3(1), dim3(dgp::CTA), lds, s, DPC); }))
      return rc;
    if (int rc = walk(e)) return rc;
    if (int rc = set_runids(e)) return rc;
  }
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
  if (hipMalloc((void**)&e->ctl, sizeof(dgp::Ctl)) != hipSuccess ||
      hipMalloc((void**)&e->d_aux, 4 * sizeof(long long)) != hipSuccess ||
      hipMalloc((void**)&e->d_dev, 2 * sizeof(dgp::Dev)) != hipSuccess) {
    (void)hipStreamDestroy(e->stream);
    delete e;
    return nullptr;
  }
  {
    namespace S = dgp::st;
    const size_t st = (size_t)S::RS * S::PLC;  // staging rows of the retire ring
    int rc = 0;
    rc |= dalloc(e, &e->D.desc, (size_t)S::DR * S::NE, e->allocs);
    rc |= dalloc(e, &e->D.dring, (size_t)S::DR * S::PX, e->allocs);
    rc |= dalloc(e, &e->D.touch_ring, (size_t)S::DR * S::TMAX, e->allocs);
    rc |= dalloc(e, &e->D.thdr, (size_t)S::DR, e->allocs);
    rc |= dalloc(e, &e->D.s2_task, st, e->allocs);
    rc |= dalloc(e, &e->D.s2_worker, st, e->allocs);
    rc |= dalloc(e, &e->D.s2_comm, st, e->allocs);
    rc |= dalloc(e, &e->D.s2_start, st, e->allocs);
    rc |= dalloc(e, &e->D.s2_wsnb, st, e->allocs);
    rc |= dalloc(e, &e->D.s2_route, st, e->allocs);
    rc |= dalloc(e, &e->D.srec, st, e->allocs);
    rc |= dalloc(e, &e->D.pos, 1, e->allocs);
    if (rc) {
      free_list(e->allocs);
      (void)hipStreamDestroy(e->stream);
      delete e;
      return nullptr;
    }
  }
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
  if (e->posted == 1) {  // a posted batch: its answer first (the kernel is inside the request)
    std::vector<int8_t> st((size_t)std::max<int64_t>(e->posted_n, 1));
    (void)resident_wait(e, st.data(), nullptr);
  }
  e->posted = 0;
  (void)resident_stop(e);
  (void)hipStreamSynchronize(e->stream);
  if (e->mb) (void)hipHostFree(e->mb);
  free_list(e->allocs);
  free_list(e->graph_allocs);
  if (e->d_msgs) (void)hipFree(e->d_msgs);
  if (e->d_status) (void)hipFree(e->d_status);
  if (e->h_msgs) (void)hipHostFree(e->h_msgs);
  if (e->d_ev) (void)hipFree(e->d_ev);
  if (e->d_msgbuf) (void)hipFree(e->d_msgbuf);
  if (e->steal.arena) (void)hipFree(e->steal.arena);
  (void)hipFree(e->ctl);
  (void)hipFree(e->d_aux);
  (void)hipFree(e->d_dev);
  if (e->d_rdy) (void)hipFree(e->d_rdy);
  for (hipEvent_t ev : e->evpool) (void)hipEventDestroy(ev);
  (void)hipStreamDestroy(e->stream);
  delete e;
}

const char* dgp_last_error(const dgp_engine* e) { return e ? e->err.c_str() : "null engine"; }

int dgp_set_config(dgp_engine* e, int64_t bandwidth, int64_t default_data_size, double unknown_duration,
                   double saturation) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e) return DGP_E_ARG;
  if (bandwidth <= 0 || default_data_size < 0 || !(saturation > 0))
    return fail(e, DGP_E_ARG, "bandwidth must be > 0, default_data_size >= 0, saturation > 0");
  e->D.bandwidth = (double)bandwidth;
  e->D.default_data_size = default_data_size;
  e->D.unknown_duration = unknown_duration;
  e->D.saturation = saturation;
  e->D.sat_inf = std::isinf(saturation) ? 1 : 0;
  e->have_config = true;
  if (e->have_workers) {  // slot caps depend on the saturation (_task_slots_available :8765)
    std::vector<int32_t> cap(e->nthreads.size());
    for (size_t w = 0; w < cap.size(); w++)
      cap[w] = e->D.sat_inf ? 0 : std::max((int32_t)std::ceil(saturation * e->nthreads[w]), (int32_t)1);
    HIPCHK(e, hipMemcpy(e->D.w_cap, cap.data(), cap.size() * 4, hipMemcpyHostToDevice));
  }
  return 0;
}

int dgp_set_workers(dgp_engine* e, int32_t n_workers, const int32_t* nthreads) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || n_workers <= 0 || !nthreads) return fail(e, DGP_E_ARG, "need n_workers > 0 and nthreads");
  if (n_workers > 32768) return fail(e, DGP_E_ARG, "at most 32768 workers (commit reservation table in LDS)");
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
  D.Wp = 1;
  while (D.Wp < n_workers) D.Wp <<= 1;
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
  rc |= dalloc(e, &D.w_lastcheck, n_workers, e->allocs);
  rc |= dalloc(e, &D.w_needs, (size_t)n_workers * dgp::NEEDS_W, e->allocs);
  {
    namespace S = dgp::st;
    const size_t W = n_workers;
    rc |= dalloc(e, &D.gw_nproc, W, e->allocs);
    rc |= dalloc(e, &D.gw_nthreads, W, e->allocs);
    rc |= dalloc(e, &D.gw_cap, W, e->allocs);
    rc |= dalloc(e, &D.gw_plen, W, e->allocs);
    rc |= dalloc(e, &D.gw_pcnt, W * S::PD, e->allocs);
    rc |= dalloc(e, &D.gw_netocc, W, e->allocs);
    rc |= dalloc(e, &D.gw_nbytes, W, e->allocs);
    rc |= dalloc(e, &D.gw_mask, W, e->allocs);
    rc |= dalloc(e, &D.gw_needs, W * S::NLW, e->allocs);
    rc |= dalloc(e, &D.gw_wflags, W, e->allocs);
    rc |= dalloc(e, &D.gw_needs_ext, W * S::NXW, e->allocs);
    rc |= dalloc(e, &D.gw_held, 2 * W, e->allocs);
    rc |= dalloc(e, &D.gw_needs_saved, W * S::NLW, e->allocs);
  }
  rc |= dalloc(e, &D.t_key, 2 * (size_t)D.Wp, e->allocs);
  rc |= dalloc(e, &D.t_idx, 2 * (size_t)D.Wp, e->allocs);
  if (rc) return DGP_E_HIP;
  HIPCHK(e, hipMemcpy(D.w_nthreads, nthreads, (size_t)n_workers * 4, hipMemcpyHostToDevice));
  e->have_workers = true;
  return dgp_set_config(e, (int64_t)D.bandwidth, D.default_data_size, D.unknown_duration, D.saturation);
}

}  // extern "C"

namespace {

// Validate a whole graph, derive its host-side structures (dependents CSR in priority order,
// priority order, root-ish groups, task flags) and upload it into fresh allocations on
// e->graph_allocs. Dynamic state is left to the caller (dgp_reset, or dgp_add_graph's copy).
int upload_graph(dgp_engine* e, int64_t n_tasks, const int64_t* dep_ptr, const int32_t* dep_idx, const int64_t* prio,
                 const int32_t* prefix_id, int32_t n_prefixes, const double* prefix_default_duration,
                 const int32_t* group_id, int32_t n_groups, const uint8_t* wanted, const int8_t* rootish_override) {
  if (n_tasks <= 0 || n_tasks >= (1ll << 24) - 1) return fail(e, DGP_E_ARG, "n_tasks out of range (< 2^24 - 1)");
  if (n_prefixes <= 0 || n_groups <= 0) return fail(e, DGP_E_ARG, "need prefixes and groups");
  if (n_prefixes > 4096) return fail(e, DGP_E_ARG, "at most 4096 task prefixes");
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
  // dependents CSR, each row in ascending priority (the frontier order of _add_to_memory)
  std::vector<int64_t> dpt_ptr(N + 1, 0);
  for (int64_t k = 0; k < E; k++) dpt_ptr[dep_idx[k] + 1]++;
  for (int64_t t = 0; t < N; t++) dpt_ptr[t + 1] += dpt_ptr[t];
  std::vector<int32_t> dpt_idx(E > 0 ? E : 1);
  {
    std::vector<int64_t> fill(dpt_ptr.begin(), dpt_ptr.end() - 1);
    for (int64_t t = 0; t < N; t++)
      for (int64_t k = dep_ptr[t]; k < dep_ptr[t + 1]; k++) dpt_idx[fill[dep_idx[k]]++] = (int32_t)t;
    for (int64_t t = 0; t < N; t++)
      if (dpt_ptr[t + 1] - dpt_ptr[t] > 1)
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
  // static is_rootish per group (:2929-2947; total_nthreads is fixed for the engine)
  std::vector<int64_t> gsize(n_groups, 0);
  for (int64_t t = 0; t < N; t++) gsize[group_id[t]]++;
  std::vector<std::vector<int32_t>> gdeps(n_groups);
  for (int64_t t = 0; t < N; t++)
    for (int64_t k = dep_ptr[t]; k < dep_ptr[t + 1]; k++) gdeps[group_id[t]].push_back(group_id[dep_idx[k]]);
  std::vector<uint8_t> grootish(n_groups, 0);
  e->gdep_n.clear();
  e->gdep_len.clear();
  for (int g = 0; g < n_groups; g++) {
    auto& v = gdeps[g];
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    int64_t sum_len = 0;
    for (int32_t d : v) sum_len += gsize[d];
    grootish[g] = (gsize[g] > e->D.total_nthreads * 2 && (int64_t)v.size() < 5 && sum_len < 5) ? 1 : 0;
    e->gdep_n.push_back((int64_t)v.size());
    e->gdep_len.push_back(sum_len);
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
  rc |= dalloc(e, &D.pdur_cur, n_prefixes, L);
  rc |= dalloc(e, &D.pdur_walk, n_prefixes, L);
  rc |= dalloc(e, &D.pdur_pre, n_prefixes, L);
  rc |= dalloc(e, &D.pmaxexec, n_prefixes, L);
  rc |= dalloc(e, &D.durv, (size_t)N * n_prefixes, L);
  rc |= dalloc(e, &D.g_size, n_groups, L);
  rc |= dalloc(e, &D.g_relwait, n_groups, L);
  rc |= dalloc(e, &D.g_left, n_groups, L);
  rc |= dalloc(e, &D.g_lastw, n_groups, L);
  rc |= dalloc(e, &D.qarr, N, L);
  // the logs: N entries (one placement / completion per task) unless a service session
  // re-placed tasks (rescheduled, recomputed): then at least what it used (grow_logs)
  D.pl_cap = std::max<int64_t>(N, e->log_min[0]);
  rc |= dalloc(e, &D.pl_task, D.pl_cap, L);
  rc |= dalloc(e, &D.pl_worker, D.pl_cap, L);
  rc |= dalloc(e, &D.pl_comm, D.pl_cap, L);
  rc |= dalloc(e, &D.pl_start, D.pl_cap, L);
  rc |= dalloc(e, &D.pl_wsnbytes, D.pl_cap, L);
  rc |= dalloc(e, &D.pl_route, D.pl_cap, L);
  int64_t capmax = 1;
  for (int32_t nt : e->nthreads) capmax = std::max<int64_t>(capmax, (int64_t)std::ceil(std::min(D.saturation, 64.0) * nt));
  D.rec_cap = 3 * N + N * std::min<int64_t>(capmax, 8) + 4096;
  rc |= dalloc(e, &D.rec, D.rec_cap, L);
  rc |= dalloc(e, &D.ev_w, N, L);
  rc |= dalloc(e, &D.ev_nf, N, L);
  rc |= dalloc(e, &D.ev_flags, N, L);
  rc |= dalloc(e, &D.ev_ntouch, N, L);
  rc |= dalloc(e, &D.ev_touch, (size_t)N * dgp::TOUCH_MAX, L);
  rc |= dalloc(e, &D.ev_plbase, N, L);
  rc |= dalloc(e, &D.ev_recbase, N, L);
  rc |= dalloc(e, &D.ev_npl, N, L);
  rc |= dalloc(e, &D.ev_pops, N, L);
  rc |= dalloc(e, &D.ev_popmax, N, L);
  D.st_cap = 2 * N + N * std::min<int64_t>(capmax, 8) + 4096;
  rc |= dalloc(e, &D.st_task, D.st_cap, L);
  rc |= dalloc(e, &D.st_worker, D.st_cap, L);
  rc |= dalloc(e, &D.st_comm, D.st_cap, L);
  rc |= dalloc(e, &D.st_start, D.st_cap, L);
  rc |= dalloc(e, &D.st_wsnbytes, D.st_cap, L);
  rc |= dalloc(e, &D.st_route, D.st_cap, L);
  rc |= dalloc(e, &D.ready, N, L);
  rc |= dalloc(e, &D.run_id, N, L);
  rc |= dalloc(e, &D.holder_of, N, L);
  rc |= dalloc(e, &D.tdyn, N, L);
  rc |= dalloc(e, &D.fr_mark, N, L);
  rc |= dalloc(e, &D.rel_mark, N, L);
  D.rlog_cap = std::max<int64_t>(2 * N + 4096, e->log_min[2]);
  rc |= dalloc(e, &D.rlog, D.rlog_cap, L);
  // service mode: the stimulus log (each task completes at most once) and its length
  D.sv_cap = std::max<int64_t>(N, e->log_min[1]);
  rc |= dalloc(e, &D.sv_task, D.sv_cap, L);
  rc |= dalloc(e, &D.sv_worker, D.sv_cap, L);
  rc |= dalloc(e, &D.sv_cseq, N, L);
  rc |= dalloc(e, &D.svc_len, 1, L);
  if (rc) return DGP_E_HIP;
  // completion reports default to "unknown" until dgp_set_task_results / dgp_tasks_finished
  HIPCHK(e, hipMemset(D.res_nbytes, 0xff, N * 8));
  HIPCHK(e, hipMemset(D.res_start, 0, N * 8));
  HIPCHK(e, hipMemset(D.res_stop, 0, N * 8));
  auto up = [&](const void* dst, const void* src, size_t bytes) {
    return hipMemcpy(const_cast<void*>(dst), src, bytes, hipMemcpyHostToDevice);
  };
  HIPCHK(e, up(D.dep_ptr, dep_ptr, (N + 1) * 8));
  if (E > 0) HIPCHK(e, up(D.dep_idx, dep_idx, E * 4));
  HIPCHK(e, up(D.dpt_ptr, dpt_ptr.data(), (N + 1) * 8));
  if (E > 0) HIPCHK(e, up(D.dpt_idx, dpt_idx.data(), E * 4));
  HIPCHK(e, up(D.prio, prio, N * 8));
  HIPCHK(e, up(D.prefix, prefix_id, N * 4));
  HIPCHK(e, up(D.group, group_id, N * 4));
  HIPCHK(e, up(D.tflags, tflags.data(), N));
  HIPCHK(e, up(D.order, order.data(), N * 4));
  HIPCHK(e, up(D.g_size, gsize.data(), n_groups * 8));
  e->prefix_defaults.assign(prefix_default_duration, prefix_default_duration + n_prefixes);
  e->group_sizes = gsize;
  e->tflags_h = tflags;
  e->group_h.assign(group_id, group_id + N);
  e->rootish_override_h.assign(rootish_override, rootish_override + N);
  e->h_dep_ptr.assign(dep_ptr, dep_ptr + N + 1);
  e->h_wide.clear();
  for (int64_t t = 0; t < N; t++)
    if (dep_ptr[t + 1] - dep_ptr[t] > dgp::UG_WIDE) e->h_wide.push_back((int32_t)t);
  e->h_dep_idx.assign(dep_idx, dep_idx + E);
  e->h_prio.assign(prio, prio + N);
  e->h_prefix.assign(prefix_id, prefix_id + N);
  e->h_wanted.assign(wanted, wanted + N);
  D.restr_ptr = nullptr;  // no restrictions until dgp_set_restrictions
  D.restr_idx = nullptr;
  D.restr_flags = nullptr;
  D.restr_ovr = nullptr;
  D.restr_pool = nullptr;
  e->rpool_used = e->rpool_cap = 0;
  e->restr_h.clear();
  return 0;
}

}  // namespace

extern "C" {

int dgp_set_graph(dgp_engine* e, int64_t n_tasks, const int64_t* dep_ptr, const int32_t* dep_idx, const int64_t* prio,
                  const int32_t* prefix_id, int32_t n_prefixes, const double* prefix_default_duration,
                  const int32_t* group_id, int32_t n_groups, const uint8_t* wanted, const int8_t* rootish_override) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e) return DGP_E_ARG;
  if (!e->have_workers) return fail(e, DGP_E_STATE, "dgp_set_workers must come first");
  HIPCHK(e, hipSetDevice(e->device));
  free_list(e->graph_allocs);
  e->have_graph = false;
  if (int rc = upload_graph(e, n_tasks, dep_ptr, dep_idx, prio, prefix_id, n_prefixes, prefix_default_duration,
                            group_id, n_groups, wanted, rootish_override))
    return rc;
  e->have_graph = true;
  e->err.clear();
  return dgp_reset(e);
}

int dgp_set_restrictions(dgp_engine* e, const int64_t* restr_ptr, const int32_t* restr_idx, const uint8_t* flags) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->have_graph) return fail(e, DGP_E_STATE, "graph first");
  if (e->mode != 0 || e->stream_used) return fail(e, DGP_E_STATE, "restrictions go with the graph, before any stimulus");
  HIPCHK(e, hipSetDevice(e->device));
  dgp::Dev& D = e->D;
  const int64_t N = D.N;
  std::vector<uint8_t> tf = e->tflags_h;
  if (flags) {
    if (!restr_ptr || restr_ptr[0] != 0) return fail(e, DGP_E_ARG, "dgp_set_restrictions: restr_ptr");
    for (int64_t t = 0; t < N; t++) {
      if (restr_ptr[t + 1] < restr_ptr[t]) return fail(e, DGP_E_ARG, "dgp_set_restrictions: restr_ptr not monotone");
      if (flags[t] & ~(dgp::RF_RESTRICTED | dgp::RF_LOOSE)) return fail(e, DGP_E_ARG, "dgp_set_restrictions: flags");
      if (!(flags[t] & dgp::RF_RESTRICTED) && restr_ptr[t + 1] != restr_ptr[t])
        return fail(e, DGP_E_ARG, "dgp_set_restrictions: valid workers on an unrestricted task");
      for (int64_t k = restr_ptr[t]; k < restr_ptr[t + 1]; k++) {
        if (restr_idx[k] < 0 || restr_idx[k] >= D.W) return fail(e, DGP_E_ARG, "dgp_set_restrictions: worker index");
        if (k > restr_ptr[t] && restr_idx[k] <= restr_idx[k - 1])
          return fail(e, DGP_E_ARG, "dgp_set_restrictions: valid workers must ascend");
      }
      // is_rootish (:2929-2947): a restricted task is not root-ish unless _rootish says so
      if ((flags[t] & dgp::RF_RESTRICTED) && e->rootish_override_h[t] < 0) tf[t] &= (uint8_t)~dgp::TF_ROOTISH;
    }
  }
  // the arrays live with the graph (freed by the next dgp_set_graph)
  int64_t* rp = nullptr;
  int32_t* ri = nullptr;
  uint8_t* rf = nullptr;
  if (flags) {
    const int64_t K = restr_ptr[N];
    int rc = 0;
    rc |= dalloc(e, &rp, N + 1, e->graph_allocs);
    rc |= dalloc(e, &ri, std::max<int64_t>(K, 1), e->graph_allocs);
    rc |= dalloc(e, &rf, N, e->graph_allocs);
    if (rc) return DGP_E_HIP;
    HIPCHK(e, hipMemcpy(rp, restr_ptr, (N + 1) * 8, hipMemcpyHostToDevice));
    if (K) HIPCHK(e, hipMemcpy(ri, restr_idx, K * 4, hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(rf, flags, N, hipMemcpyHostToDevice));
  }
  HIPCHK(e, hipMemcpy(const_cast<uint8_t*>(D.tflags), tf.data(), N, hipMemcpyHostToDevice));
  e->tflags_h = tf;
  D.restr_ptr = rp;
  D.restr_idx = ri;
  D.restr_flags = rf;
  D.restr_ovr = nullptr;  // the new rows replace every earlier update
  D.restr_pool = nullptr;
  e->rpool_used = e->rpool_cap = 0;
  if (flags) e->restr_h.assign(flags, flags + N);
  else e->restr_h.clear();
  return dgp_reset(e);
}

namespace {
__global__ void k_restr_scatter(int64_t* ovr, uint8_t* rf, const int32_t* task, const int64_t* off, const uint8_t* fl,
                                int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    ovr[task[i]] = off[i];
    rf[task[i]] = fl[i];
  }
}
}  // namespace

int dgp_update_restrictions(dgp_engine* e, int64_t n, const int32_t* task, const int64_t* row_ptr,
                            const int32_t* row_idx, const uint8_t* flags) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->have_graph) return fail(e, DGP_E_STATE, "graph first");
  // (while an appended graph's stimulus is pending: its tasks' rows go in before dgp_graph_stimulus)
  if (n < 0 || (n && (!task || !row_ptr || !flags)) || (n && row_ptr[0] != 0))
    return fail(e, DGP_E_ARG, "dgp_update_restrictions: arguments");
  HIPCHK(e, hipSetDevice(e->device));
  dgp::Dev& D = e->D;
  const int64_t N = D.N;
  for (int64_t i = 0; i < n; i++) {
    if (task[i] < 0 || task[i] >= N) return fail(e, DGP_E_ARG, "dgp_update_restrictions: task index");
    if (flags[i] & ~(dgp::RF_RESTRICTED | dgp::RF_LOOSE)) return fail(e, DGP_E_ARG, "dgp_update_restrictions: flags");
    if (row_ptr[i + 1] < row_ptr[i]) return fail(e, DGP_E_ARG, "dgp_update_restrictions: row_ptr not monotone");
    if (!(flags[i] & dgp::RF_RESTRICTED) && row_ptr[i + 1] != row_ptr[i])
      return fail(e, DGP_E_ARG, "dgp_update_restrictions: valid workers on an unrestricted task");
    for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; k++) {
      if (row_idx[k] < 0 || row_idx[k] >= D.W) return fail(e, DGP_E_ARG, "dgp_update_restrictions: worker index");
      if (k > row_ptr[i] && row_idx[k] <= row_idx[k - 1])
        return fail(e, DGP_E_ARG, "dgp_update_restrictions: valid workers must ascend");
    }
  }
  if (n == 0) return 0;
  auto& A = e->graph_allocs;  // the arrays live with the graph
  if (!D.restr_flags) {  // the graph had none: every other task keeps an empty CSR row
    int64_t* rp = nullptr;
    int32_t* ri = nullptr;
    uint8_t* rf = nullptr;
    if (dalloc(e, &rp, N + 1, A) || dalloc(e, &ri, 1, A) || dalloc(e, &rf, N, A)) return DGP_E_HIP;
    HIPCHK(e, hipMemset(rp, 0, (N + 1) * 8));
    HIPCHK(e, hipMemset(rf, 0, N));
    D.restr_ptr = rp;
    D.restr_idx = ri;
    D.restr_flags = rf;
    e->restr_h.assign(N, 0);
  }
  if (!D.restr_ovr) {
    int64_t* ov = nullptr;
    if (dalloc(e, &ov, N, A)) return DGP_E_HIP;
    HIPCHK(e, hipMemset(ov, 0xff, N * 8));  // -1: the CSR row
    D.restr_ovr = ov;
  }
  // the rows, appended to the pool (length, then the workers)
  const int64_t add = n + row_ptr[n];
  if (e->rpool_used + add > e->rpool_cap) {
    const int64_t cap = std::max<int64_t>(std::max<int64_t>(2 * e->rpool_cap, e->rpool_used + add), 4096);
    int32_t* np = nullptr;
    if (dalloc(e, &np, cap, A)) return DGP_E_HIP;
    if (e->rpool_used) HIPCHK(e, hipMemcpy(np, D.restr_pool, e->rpool_used * 4, hipMemcpyDeviceToDevice));
    D.restr_pool = np;  // (the old pool is freed with the graph)
    e->rpool_cap = cap;
  }
  std::vector<int32_t> rows((size_t)add);
  std::vector<int64_t> off((size_t)n);
  std::vector<uint8_t> fl(flags, flags + n);
  int64_t q = 0;
  std::vector<uint8_t> tf = e->tflags_h;
  for (int64_t i = 0; i < n; i++) {
    off[i] = e->rpool_used + q;
    rows[q++] = (int32_t)(row_ptr[i + 1] - row_ptr[i]);
    for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; k++) rows[q++] = row_idx[k];
    const int t = task[i];
    e->restr_h[t] = flags[i];
    // is_rootish (:2929-2947): restrictions make a task non-root-ish unless _rootish says so
    if (e->rootish_override_h[t] < 0) {
      const int g = e->group_h[t];
      const bool gr = e->group_sizes[g] > D.total_nthreads * 2 && e->gdep_n[g] < 5 && e->gdep_len[g] < 5;
      const bool r = gr && !(flags[i] & dgp::RF_RESTRICTED);
      tf[t] = (uint8_t)((tf[t] & ~dgp::TF_ROOTISH) | (r ? dgp::TF_ROOTISH : 0));
    }
  }
  HIPCHK(e, hipMemcpy(const_cast<int32_t*>(D.restr_pool) + e->rpool_used, rows.data(), add * 4, hipMemcpyHostToDevice));
  e->rpool_used += add;
  int32_t* d_task = nullptr;
  int64_t* d_off = nullptr;
  uint8_t* d_fl = nullptr;
  std::vector<void*> tmp;
  if (dalloc(e, &d_task, n, tmp) || dalloc(e, &d_off, n, tmp) || dalloc(e, &d_fl, n, tmp)) {
    free_list(tmp);
    return DGP_E_HIP;
  }
  hipError_t st = hipMemcpy(d_task, task, n * 4, hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice);
  if (st == hipSuccess) st = hipMemcpy(d_fl, fl.data(), n, hipMemcpyHostToDevice);
  if (st == hipSuccess) {
    hipLaunchKernelGGL(k_restr_scatter, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 1024)), dim3(256), 0,
                       e->stream, const_cast<int64_t*>(D.restr_ovr), const_cast<uint8_t*>(D.restr_flags), d_task,
                       d_off, d_fl, n);
    st = hipGetLastError();
  }
  if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
  free_list(tmp);
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("dgp_update_restrictions: ") + hipGetErrorString(st));
  if (tf != e->tflags_h) {
    HIPCHK(e, hipMemcpy(const_cast<uint8_t*>(D.tflags), tf.data(), N, hipMemcpyHostToDevice));
    e->tflags_h = tf;
  }
  return 0;
}

int dgp_set_rootish(dgp_engine* e, int64_t n, const int32_t* task, const int8_t* value) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->have_graph) return fail(e, DGP_E_STATE, "graph first");
  // (while an appended graph's stimulus is pending: its tasks' flags go in before dgp_graph_stimulus)
  if (n < 0 || (n && (!task || !value))) return fail(e, DGP_E_ARG, "dgp_set_rootish: arguments");
  HIPCHK(e, hipSetDevice(e->device));
  dgp::Dev& D = e->D;
  for (int64_t i = 0; i < n; i++) {
    if (task[i] < 0 || task[i] >= D.N) return fail(e, DGP_E_ARG, "dgp_set_rootish: task index");
    if (value[i] < -1 || value[i] > 1) return fail(e, DGP_E_ARG, "dgp_set_rootish: value");
  }
  std::vector<uint8_t> tf = e->tflags_h;
  for (int64_t i = 0; i < n; i++) {  // is_rootish (:2929-2947) with the new TaskState._rootish
    const int t = task[i];
    e->rootish_override_h[t] = value[i];
    const int g = e->group_h[t];
    const bool gr = e->group_sizes[g] > D.total_nthreads * 2 && e->gdep_n[g] < 5 && e->gdep_len[g] < 5;
    const bool rs = !e->restr_h.empty() && (e->restr_h[t] & dgp::RF_RESTRICTED);
    const bool r = value[i] >= 0 ? value[i] != 0 : (gr && !rs);
    tf[t] = (uint8_t)((tf[t] & ~dgp::TF_ROOTISH) | (r ? dgp::TF_ROOTISH : 0));
  }
  if (tf != e->tflags_h) {
    HIPCHK(e, hipMemcpy(const_cast<uint8_t*>(D.tflags), tf.data(), D.N, hipMemcpyHostToDevice));
    e->tflags_h = tf;
  }
  return 0;
}

int dgp_set_task_results(dgp_engine* e, const int64_t* nbytes, const double* start, const double* stop) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->have_graph) return fail(e, DGP_E_STATE, "graph first");
  HIPCHK(e, hipSetDevice(e->device));
  size_t N = e->D.N;
  HIPCHK(e, hipMemcpy(e->D.res_nbytes, nbytes, N * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(e->D.res_start, start, N * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(e->D.res_stop, stop, N * 8, hipMemcpyHostToDevice));
  e->have_results = true;
  return 0;
}

int dgp_reset(dgp_engine* e) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->have_graph) return fail(e, DGP_E_STATE, "graph first");
  HIPCHK(e, hipSetDevice(e->device));
  dgp::Dev& D = e->D;
  const size_t N = D.N;
  hipStream_t s = e->stream;
  HIPCHK(e, hipMemsetAsync(e->ctl, 0, sizeof(dgp::Ctl), s));
  HIPCHK(e, hipMemsetAsync(e->d_aux, 0, 4 * sizeof(long long), s));
  HIPCHK(e, hipMemsetAsync(D.state, 0, N, s));
  HIPCHK(e, hipMemsetAsync(D.remaining, 0, N * 4, s));
  HIPCHK(e, hipMemsetAsync(D.waiters, 0, N * 4, s));
  HIPCHK(e, hipMemsetAsync(D.proc_on, 0xff, N * 4, s));
  HIPCHK(e, hipMemsetAsync(D.cur_nbytes, 0xff, N * 8, s));
  HIPCHK(e, hipMemsetAsync(D.holders, 0, N * D.WB * 8, s));
  HIPCHK(e, hipMemsetAsync(D.ready_key, 0, N * 8, s));
  HIPCHK(e, hipMemsetAsync(D.release_key, 0, N * 8, s));
  HIPCHK(e, hipMemsetAsync(D.cand_n, 0, N * 4, s));
  {  // stream engine
    namespace S = dgp::st;
    HIPCHK(e, hipMemsetAsync(D.run_id, 0xff, N * 4, s));
    HIPCHK(e, hipMemsetAsync(D.holder_of, 0xff, N * 4, s));
    HIPCHK(e, hipMemsetAsync(D.tdyn, 0, N, s));
    D.evf = 0;
    e->paused_h.assign(D.W, 0);
    HIPCHK(e, hipMemsetAsync(D.fr_mark, 0xff, N * 4, s));
    HIPCHK(e, hipMemsetAsync(D.rel_mark, 0xff, N * 4, s));
    HIPCHK(e, hipMemsetAsync(D.thdr, 0, (size_t)S::DR * sizeof(uint2), s));
    HIPCHK(e, hipMemsetAsync(D.gw_needs_ext, 0, (size_t)D.W * S::NXW * 4, s));
    HIPCHK(e, hipMemsetAsync(D.gw_needs_saved, 0, (size_t)D.W * S::NLW * 4, s));
    S::Pos p0{};
    p0.round_end = -1;
    HIPCHK(e, hipMemcpyAsync(D.pos, &p0, sizeof p0, hipMemcpyHostToDevice, s));
    e->stream_used = false;
    HIPCHK(e, hipMemsetAsync(D.svc_len, 0, sizeof(long long), s));
    HIPCHK(e, hipMemsetAsync(D.sv_cseq, 0xff, N * 4, s));
    e->mode = 0;
    e->last_placed = 0;
    e->sv_used = 0;
  }
  std::vector<double> maxexec(D.P, -1.0);
  HIPCHK(e, hipMemcpyAsync(D.pdur_cur, e->prefix_defaults.data(), D.P * 8, hipMemcpyHostToDevice, s));
  HIPCHK(e, hipMemcpyAsync(D.pdur_walk, e->prefix_defaults.data(), D.P * 8, hipMemcpyHostToDevice, s));
  HIPCHK(e, hipMemcpyAsync(D.pdur_pre, e->prefix_defaults.data(), D.P * 8, hipMemcpyHostToDevice, s));
  HIPCHK(e, hipMemcpyAsync(D.pmaxexec, maxexec.data(), D.P * 8, hipMemcpyHostToDevice, s));
  HIPCHK(e, hipMemcpyAsync(D.g_relwait, e->group_sizes.data(), D.G * 8, hipMemcpyHostToDevice, s));
  HIPCHK(e, hipMemsetAsync(D.g_left, 0, D.G * 8, s));
  HIPCHK(e, hipMemsetAsync(D.g_lastw, 0xff, D.G * 4, s));
  if (int rc = sync_dev(e)) return rc;
  hipLaunchKernelGGL(dgp::k_init_workers, dim3(grid_for(D.W, 256, 256)), dim3(256), 0, s, e->d_dev);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipStreamSynchronize(s));
  e->graph_done = false;
  e->evused = 0;
  for (int k = 0; k < 8; k++) {
    e->kms[k] = 0;
    e->klaunch[k] = 0;
  }
  return 0;
}

int dgp_update_graph(dgp_engine* e) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->have_graph || !e->have_config) return fail(e, DGP_E_STATE, "config, workers and graph first");
  if (e->graph_done) return fail(e, DGP_E_STATE, "update_graph already ran (dgp_reset first)");
  HIPCHK(e, hipSetDevice(e->device));
  if (int rc = sync_dev(e)) return rc;
  const dgp::Dev* DP = e->d_dev;
  hipStream_t s = e->stream;
  if (int rc = timed_launch(e, 3, [&] {
        launch_ug_init(e, 0);
      }))
    return rc;
  if (int rc = launch_ug_dispatch(e, 0, 0)) return rc;
  if (e->snap_rounds > 0) {
    hipLaunchKernelGGL(dgp::k_snapshot, dim3(8), dim3(256), 0, s, DP, e->d_aux + 1, 0);
    HIPCHK(e, hipGetLastError());
  }
  if (int rc = set_runids(e)) return rc;
  e->graph_done = true;
  // dgp_tasks_finished counts its new placements from here
  dgp::Ctl c;
  if (int rc = read_ctl(e, &c)) return rc;
  e->last_placed = c.n_placed;
  return 0;
}

int dgp_run_rounds(dgp_engine* e, int64_t max_rounds, int64_t* n_rounds_out) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (!e->have_results) return fail(e, DGP_E_STATE, "dgp_set_task_results first");
  if (e->mode == 2) return fail(e, DGP_E_STATE, "engine is in service mode (dgp_tasks_finished); dgp_reset first");
  HIPCHK(e, hipSetDevice(e->device));
  e->mode = 1;
  stream_source(e, false);
  if (n_rounds_out) *n_rounds_out = 0;
  if (max_rounds == 0) return 0;
  if (int rc = sync_dev(e)) return rc;
  dgp::Ctl c;
  if (int rc = check_device_error(e, &c)) return rc;
  const long long r0 = c.rounds_nonempty;
  const dgp::Dev& D = e->D;
  if (D.P <= dgp::st::PX) {
    // the stream engine: the whole replay in one persistent workgroup (dgp_stream.h)
    if (int rc = launch_stream(e, max_rounds, e->snap_rounds > 0 ? 1 : 0)) return rc;
  } else {
    // more task prefixes than the stream descriptors carry, or worker restrictions (decided
    // by the global dispatch, dgp_device.h OP_RESTRICTED): the round-kernel engine
    if (e->stream_used) return fail(e, DGP_E_STATE, "engine already advanced by the stream replay");
    const int lds_workers = D.W <= dgp::LDS_WORKERS_MAX ? 1 : 0;
    const size_t lds = (((size_t)D.W * sizeof(int) + 15) & ~(size_t)15) +
                       (lds_workers ? (((size_t)D.W + 3) & ~(size_t)3) * dgp::LDS_WORKER_BYTES + 64 : 0);
    if (lds + kernel_static_lds((const void*)dgp::k_replay, 0) > 160 * 1024)
      return fail(e, DGP_E_ARG, "commit LDS exceeds 160 KiB");
    const dgp::Dev* DPC = e->d_dev + 1;
    const int snaps = e->snap_rounds > 0 ? 1 : 0;
    if (int rc = timed_launch(e, 2, [&] {
          hipLaunchKernelGGL(dgp::k_replay, dim3(1), dim3(dgp::CTA), lds, e->stream, DPC, e->d_aux, (long long)max_rounds,
                             e->d_aux + 1, snaps);
        }))
      return rc;
    if (int rc = walk(e)) return rc;
  }
  if (int rc = check_device_error(e, &c)) return rc;
  if (n_rounds_out) *n_rounds_out = c.rounds_nonempty - r0;
  return 0;
}

}  // extern "C"

namespace {

// dgp_tasks_finished through the resident stream kernel: the batch goes into the pinned
// mailbox, the request number is published, and the kernel's sequencer answers it (the
// message checks, every stimulus it accepts run to completion, the new placements copied
// back); the host only spins on the answer. A kernel that ended on its own (no request for
// a while) or never started is launched first; the logs grow with the kernel stopped.
// resident_post returns as soon as the request is published (dgp_tasks_finished_post: the
// caller's own work overlaps the device's), resident_wait takes the answer.
int resident_launch(dgp_engine* e) {
  dgp::Dev& D = e->D;
  if (int rc = sync_dev(e)) return rc;
  stream_source(e, true);
  D.resident = 1;
  D.mbox = (void*)e->mb_dev;
  if (int rc = launch_stream(e, -1, 0)) {
    D.resident = 0;
    return rc;
  }
  e->res_running = true;
  return 0;
}

int resident_post(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker, const int64_t* run_id,
                  const int64_t* nbytes, const double* start, const double* stop) {
  namespace V = dgp::svc;
  dgp::Dev& D = e->D;
  const int64_t plc = std::min<int64_t>(std::max<int64_t>(D.N, 1024), 1 << 20);
  if (!e->mb || e->mb->cap < n || e->mb->pl_cap < plc) {  // the mailbox, sized for this batch
    if (int rc = resident_stop(e)) return rc;
    if (e->mb) (void)hipHostFree(e->mb);
    e->mb = nullptr;
    const int64_t cap = std::max<int64_t>(n, 4096);
    const int64_t mpc = std::min<int64_t>(plc, 65536), mdc = 8 * mpc;  // message fields: placements, entries
    void* p = nullptr;
    HIPCHK(e, hipHostMalloc(&p, V::mbox_bytes(cap, plc, mpc, mdc), hipHostMallocCoherent | hipHostMallocMapped));
    memset(p, 0, sizeof(V::Mbox));  // the whole header (t_role included)
    e->mb = (V::Mbox*)p;
    e->mb->cap = cap;
    e->mb->pl_cap = plc;
    e->mb->mp_cap = mpc;
    e->mb->md_cap = mdc;
    e->mb->msg_from = -1;
    e->mb->req_seq = e->mb->done_seq = e->req_seq;
    void* pd = nullptr;
    HIPCHK(e, hipHostGetDevicePointer(&pd, p, 0));
    e->mb_dev = (V::Mbox*)pd;
  }
  // log capacity for up to every task placed once more and n completions (grow_logs), with
  // the kernel stopped when an array must grow
  if ((int64_t)e->last_placed + D.N + 64 > D.pl_cap || e->sv_used + n > D.sv_cap) {
    if (int rc = resident_stop(e)) return rc;
    if (int rc = grow_logs(e, n)) return rc;
  }
  V::Msg* M = V::mbox_msgs(e->mb);
  for (int64_t i = 0; i < n; i++) M[i] = V::Msg{task[i], worker[i], run_id[i], nbytes[i], start[i], stop[i]};
  e->mb->n = n;
  e->mb->want_msgs = e->res_msgs ? 1 : 0;
  e->mb->msg_from = -1;
  if (!e->res_running)
    if (int rc = resident_launch(e)) return rc;
  const unsigned long long seq = ++e->req_seq;
  __atomic_store_n(&e->mb->req_seq, seq, __ATOMIC_RELEASE);
  e->posted = 1;
  e->posted_n = n;
  return 0;
}

int resident_wait(dgp_engine* e, int8_t* status, int64_t* n_new_placements) {
  namespace V = dgp::svc;
  dgp::Dev& D = e->D;
  const int64_t n = e->posted_n;
  const unsigned long long seq = e->req_seq;
  e->posted = 0;  // answered or failed below: the engine's other entry points are open again
  const auto t0 = std::chrono::steady_clock::now();
  for (long spins = 0; __atomic_load_n(&e->mb->done_seq, __ATOMIC_ACQUIRE) != seq; spins++) {
    if ((spins & 255) == 255) {
      if (hipStreamQuery(e->stream) == hipSuccess) {  // the kernel ended: idle before this request, or an error
        e->res_running = false;
        D.resident = 0;
        if (int rc = check_device_error(e)) return rc;
        if (__atomic_load_n(&e->mb->done_seq, __ATOMIC_ACQUIRE) == seq) break;
        if (int rc = resident_launch(e)) return rc;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
        // told to stop, waited for a bounded time (a kernel stuck inside a request never
        // reads the flag): never a blocking synchronisation here
        __atomic_store_n(&e->mb->stop, 1, __ATOMIC_RELEASE);
        const auto t1 = std::chrono::steady_clock::now();
        hipError_t q = hipStreamQuery(e->stream);
        while (q == hipErrorNotReady && std::chrono::steady_clock::now() - t1 < std::chrono::seconds(5)) {
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
          q = hipStreamQuery(e->stream);
        }
        if (q == hipErrorNotReady) {
          e->res_hung = true;
        } else {
          __atomic_store_n(&e->mb->stop, 0, __ATOMIC_RELEASE);
          e->res_running = false;
          D.resident = 0;
        }
        return fail(e, DGP_E_DEVICE, "dgp_tasks_finished: the resident kernel did not answer within 60 s");
      }
    }
  }
  if (e->mb->error) {  // the kernel ends on a device error: report it from the control block
    if (int rc = resident_stop(e)) return rc;
    if (int rc = check_device_error(e)) return rc;
  }
  memcpy(status, V::mbox_status(e->mb), (size_t)n);
  e->res_prof[0] += 1;
  if (e->mb->t_app >= e->mb->t_seen && e->mb->t_ret >= e->mb->t_app && e->mb->t_pub >= e->mb->t_ret) {
    e->res_prof[1] += (int64_t)(e->mb->t_app - e->mb->t_seen);
    e->res_prof[2] += (int64_t)(e->mb->t_ret - e->mb->t_app);
    e->res_prof[3] += (int64_t)(e->mb->t_pub - e->mb->t_ret);
    for (int k = 0; k < 7; k++)
      if (e->mb->t_role[k] >= e->mb->t_app && e->mb->t_role[k] <= e->mb->t_pub)
        e->res_role[k] += (int64_t)(e->mb->t_role[k] - e->mb->t_app);
  }
  const unsigned long long placed = (unsigned long long)e->mb->n_placed;
  if (n_new_placements) *n_new_placements = (int64_t)(placed - e->last_placed);
  e->last_placed = placed;
  for (int64_t i = 0; i < n; i++) e->sv_used += status[i] == DGP_TF_ACCEPTED ? 1 : 0;
  return 0;
}

}  // namespace

extern "C" {

int dgp_set_task_messages(dgp_engine* e, int enabled) {
  if (!e) return DGP_E_ARG;
  e->res_msgs = enabled != 0;
  return 0;
}

int dgp_set_resident(dgp_engine* e, int enabled) {
  if (!e) return DGP_E_ARG;
  if (!enabled)
    if (int rc = resident_stop(e)) return rc;
  e->resident = enabled != 0;
  return 0;
}

}  // extern "C"

namespace {

// the preconditions of dgp_tasks_finished / dgp_tasks_finished_post
int tf_check(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker, const int64_t* run_id,
             const int64_t* nbytes, const double* start, const double* stop) {
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (e->posted) return fail(e, DGP_E_STATE, "a posted task-finished batch: dgp_tasks_finished_wait first");
  if (e->mode == 1) return fail(e, DGP_E_STATE, "engine advanced by a replay (dgp_run_rounds); dgp_reset first");
  if (e->pending_resync) return fail(e, DGP_E_STATE, "dgp_tasks_finished: dgp_sync_* first (a later graph depends on earlier tasks)");
  if (n < 0 || (n > 0 && (!task || !worker || !run_id || !nbytes || !start || !stop)))
    return fail(e, DGP_E_ARG, "dgp_tasks_finished: bad batch");
  HIPCHK(e, hipSetDevice(e->device));
  e->mode = 2;
  return 0;
}

bool tf_resident(const dgp_engine* e) { return e->resident && e->D.P <= dgp::st::PX; }

// dgp_tasks_finished launched per call: the batch copied to the device, the service kernels,
// the answers copied back
int tasks_finished_launch(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker,
                          const int64_t* run_id, const int64_t* nbytes, const double* start, const double* stop,
                          int8_t* status, int64_t* n_new_placements) {
  if (int rc = resident_stop(e)) return rc;
  namespace V = dgp::svc;
  if (n > e->msgs_cap) {  // grow the pinned staging and the device batch
    if (e->d_msgs) (void)hipFree(e->d_msgs);
    if (e->d_status) (void)hipFree(e->d_status);
    if (e->h_msgs) (void)hipHostFree(e->h_msgs);
    e->d_msgs = nullptr;
    e->d_status = nullptr;
    e->h_msgs = nullptr;
    e->msgs_cap = 0;
    const int64_t cap = std::max<int64_t>(n, 1024);
    HIPCHK(e, hipMalloc((void**)&e->d_msgs, cap * sizeof(V::Msg)));
    HIPCHK(e, hipMalloc((void**)&e->d_status, cap));
    HIPCHK(e, hipHostMalloc((void**)&e->h_msgs, cap * sizeof(V::Msg), hipHostMallocDefault));
    e->msgs_cap = cap;
  }
  for (int64_t i = 0; i < n; i++) e->h_msgs[i] = V::Msg{task[i], worker[i], run_id[i], nbytes[i], start[i], stop[i]};
  hipStream_t s = e->stream;
  if (int rc = grow_logs(e, n)) return rc;
  if (int rc = sync_dev(e)) return rc;
  HIPCHK(e, hipMemcpyAsync(e->d_msgs, e->h_msgs, n * sizeof(V::Msg), hipMemcpyHostToDevice, s));
  // the batch in segments: each ends where an answer depends on the segment's own stimuli
  // (k_svc_append); usually the whole batch is one segment
  long long* d_consumed = e->d_aux + 3;
  dgp::Ctl c;
  for (int64_t off = 0; off < n;) {
    hipLaunchKernelGGL(V::k_svc_append, dim3(1), dim3(64), 0, s, e->d_dev, e->d_msgs + off, (long long)(n - off),
                       e->d_status + off, d_consumed);
    HIPCHK(e, hipGetLastError());
    if (int rc = run_service_stimuli(e)) return rc;
    long long k = 0;
    HIPCHK(e, hipMemcpyAsync(&k, d_consumed, sizeof k, hipMemcpyDeviceToHost, s));
    // the answers so far ride on the same synchronisation (the last segment's are final)
    HIPCHK(e, hipMemcpyAsync(status, e->d_status, n, hipMemcpyDeviceToHost, s));
    if (int rc = check_device_error(e, &c)) return rc;  // synchronises the stream
    if (k <= 0) return fail(e, DGP_E_DEVICE, "dgp_tasks_finished: no progress on the batch");
    off += k;
  }
  if (n_new_placements) *n_new_placements = (int64_t)(c.n_placed - e->last_placed);
  e->last_placed = c.n_placed;
  for (int64_t i = 0; i < n; i++) e->sv_used += status[i] == DGP_TF_ACCEPTED ? 1 : 0;
  return 0;
}

}  // namespace

extern "C" {

int dgp_tasks_finished(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker, const int64_t* run_id,
                       const int64_t* nbytes, const double* start, const double* stop, int8_t* status,
                       int64_t* n_new_placements) {
  if (int rc = tf_check(e, n, task, worker, run_id, nbytes, start, stop)) return rc;
  if (n > 0 && !status) return fail(e, DGP_E_ARG, "dgp_tasks_finished: bad batch");
  if (n_new_placements) *n_new_placements = 0;
  if (n == 0) return 0;
  if (tf_resident(e)) {
    if (int rc = resident_post(e, n, task, worker, run_id, nbytes, start, stop)) return rc;
    return resident_wait(e, status, n_new_placements);
  }
  return tasks_finished_launch(e, n, task, worker, run_id, nbytes, start, stop, status, n_new_placements);
}

int dgp_tasks_finished_post(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker,
                            const int64_t* run_id, const int64_t* nbytes, const double* start, const double* stop) {
  if (int rc = tf_check(e, n, task, worker, run_id, nbytes, start, stop)) return rc;
  if (n > 0 && tf_resident(e)) return resident_post(e, n, task, worker, run_id, nbytes, start, stop);
  // launch per call: answered here, kept for the wait
  e->posted_status.assign((size_t)std::max<int64_t>(n, 1), 0);
  e->posted_new = 0;
  if (n > 0)
    if (int rc = tasks_finished_launch(e, n, task, worker, run_id, nbytes, start, stop, e->posted_status.data(),
                                       &e->posted_new))
      return rc;
  e->posted = 2;
  e->posted_n = n;
  return 0;
}

int dgp_tasks_finished_wait(dgp_engine* e, int8_t* status, int64_t* n_new_placements) {
  if (!e) return DGP_E_ARG;
  if (!e->posted) return fail(e, DGP_E_STATE, "dgp_tasks_finished_wait: no batch posted");
  if (e->posted_n > 0 && !status) return fail(e, DGP_E_ARG, "dgp_tasks_finished_wait: no status array");
  if (n_new_placements) *n_new_placements = 0;
  if (e->posted == 1) return resident_wait(e, status, n_new_placements);
  if (e->posted_n > 0) memcpy(status, e->posted_status.data(), (size_t)e->posted_n);
  if (n_new_placements) *n_new_placements = e->posted_new;
  e->posted = 0;
  return 0;
}

int dgp_set_window(dgp_engine* e, int32_t window) {
  if (!e) return DGP_E_ARG;
  if (window != 32 && window != 64) return fail(e, DGP_E_ARG, "dgp_set_window: window must be 32 or 64");
  if (int rc_ = resident_stop(e)) return rc_;  // the next launch takes the other build
  e->window = window;
  return 0;
}

int dgp_get_window(dgp_engine* e) { return e ? e->window : 0; }

int dgp_move_task(dgp_engine* e, int32_t task, int32_t thief) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (e->mode == 1) return fail(e, DGP_E_STATE, "engine advanced by a replay (dgp_run_rounds); dgp_reset first");
  if (!(e->D.P <= dgp::st::PX))
    return fail(e, DGP_E_STATE, "dgp_move_task: the round-kernel engine (more than 32 prefixes) "
                                "has no steal confirmation");
  if (e->pending_resync) return fail(e, DGP_E_STATE, "dgp_move_task: dgp_sync_* first (a later graph depends on earlier tasks)");
  if (task < 0 || task >= e->D.N || thief < 0 || thief >= e->D.W)
    return fail(e, DGP_E_ARG, "dgp_move_task: task or thief out of range");
  HIPCHK(e, hipSetDevice(e->device));
  e->mode = 2;
  if (int rc = sync_dev(e)) return rc;
  hipLaunchKernelGGL(dgp::st::k_move_task, dim3(1), dim3(64), 0, e->stream, e->d_dev, task, thief);
  HIPCHK(e, hipGetLastError());
  return check_device_error(e);
}

}  // extern "C"

namespace {
// a worker inserted at index pos: every worker index >= pos held per task moves up by one
// (holder_of, processing_on) and each who_has bitset row gains a zero bit at pos
__global__ void k_insert_worker_remap(int32_t* holder_of, int32_t* proc_on, unsigned long long* holders, int64_t N,
                                      int32_t WB, int32_t pos) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < N; t += (int64_t)gridDim.x * blockDim.x) {
    if (holder_of[t] >= pos) holder_of[t] += 1;
    if (proc_on[t] >= pos) proc_on[t] += 1;
    unsigned long long* row = holders + (size_t)t * WB;
    const int k0 = pos >> 6, b0 = pos & 63;
    const unsigned long long low = b0 ? ((1ull << b0) - 1) : 0ull;  // bits below pos stay
    unsigned long long carry = 0;  // the top bit of the previous word, moving into this one
    for (int k = k0; k < WB; k++) {
      const unsigned long long v = row[k];
      row[k] = k == k0 ? ((v & low) | ((v & ~low) << 1)) : ((v << 1) | carry);
      carry = v >> 63;
    }
  }
}
__global__ void k_remap_range(int32_t* a, int64_t n, int32_t pos) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (a[i] >= pos) a[i] += 1;
}
}  // namespace

extern "C" {

int dgp_add_worker(dgp_engine* e, int32_t nthreads, int64_t* n_new_placements) {
  return dgp_add_worker_at(e, nthreads, 1, e ? e->D.W : 0, n_new_placements);
}

int dgp_add_worker_at(dgp_engine* e, int32_t nthreads, int32_t running, int32_t position, int64_t* n_new_placements) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (n_new_placements) *n_new_placements = 0;
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (e->mode == 1) return fail(e, DGP_E_STATE, "engine advanced by a replay (dgp_run_rounds); dgp_reset first");
  if (e->pending_resync) return fail(e, DGP_E_STATE, "dgp_add_worker: dgp_sync_* first (a later graph depends on earlier tasks)");
  if (!(e->D.P <= dgp::st::PX))
    return fail(e, DGP_E_STATE, "dgp_add_worker: the round-kernel engine (more than 32 prefixes) "
                                "has no worker addition");
  if (nthreads <= 0 || nthreads > 65535) return fail(e, DGP_E_ARG, "dgp_add_worker: nthreads out of range");
  if (e->D.W + 1 > 32768) return fail(e, DGP_E_ARG, "at most 32768 workers");
  if (position < 0 || position > e->D.W) return fail(e, DGP_E_ARG, "dgp_add_worker_at: position out of range");
  {  // no-worker tasks would be rescheduled on the new worker (bulk_schedule_unrunnable_after_adding_worker)
    dgp::Ctl c;
    if (int rc = read_ctl(e, &c)) return rc;
    if (c.n_unrunnable > 0)
      return fail(e, DGP_E_STATE, "dgp_add_worker: no-worker tasks would be rescheduled (not modelled)");
  }
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (position < e->D.W) {  // the stream positions must be settled: no descriptor or record waits with old indices
    dgp::st::Pos ps;
    HIPCHK(e, hipMemcpy(&ps, e->D.pos, sizeof ps, hipMemcpyDeviceToHost));
    if (ps.pre > ps.seq || ps.walk != ps.rec_len)
      return fail(e, DGP_E_STATE, "dgp_add_worker_at: the stream engine has prefetched stimuli or unfolded records");
  }
  namespace S = dgp::st;
  dgp::Dev& D = e->D;
  const size_t W0 = D.W, W1 = W0 + 1;
  auto& A = e->allocs;
  int rc = 0;
  // every per-worker array one row longer (rows are per worker: a prefix copy)
  rc |= regrow(e, &D.w_nthreads, W0, W1, A);
  rc |= regrow(e, &D.w_cap, W0, W1, A);
  rc |= regrow(e, &D.w_nproc, W0, W1, A);
  rc |= regrow(e, &D.w_plen, W0, W1, A);
  rc |= regrow(e, &D.w_pfx, W0 * dgp::PMAX, W1 * dgp::PMAX, A);
  rc |= regrow(e, &D.w_pcnt, W0 * dgp::PMAX, W1 * dgp::PMAX, A);
  rc |= regrow(e, &D.w_netocc, W0, W1, A);
  rc |= regrow(e, &D.w_nbytes, W0, W1, A);
  rc |= regrow(e, &D.w_flags, W0, W1, A);
  rc |= regrow(e, &D.w_itcslots, W0, W1, A);
  rc |= regrow(e, &D.w_lastcheck, W0, W1, A);
  rc |= regrow(e, &D.w_needs, W0 * dgp::NEEDS_W, W1 * dgp::NEEDS_W, A);
  rc |= regrow(e, &D.gw_nproc, W0, W1, A);
  rc |= regrow(e, &D.gw_nthreads, W0, W1, A);
  rc |= regrow(e, &D.gw_cap, W0, W1, A);
  rc |= regrow(e, &D.gw_plen, W0, W1, A);
  rc |= regrow(e, &D.gw_pcnt, W0 * S::PD, W1 * S::PD, A);
  rc |= regrow(e, &D.gw_netocc, W0, W1, A);
  rc |= regrow(e, &D.gw_nbytes, W0, W1, A);
  rc |= regrow(e, &D.gw_mask, W0, W1, A);
  rc |= regrow(e, &D.gw_needs, W0 * S::NLW, W1 * S::NLW, A);
  rc |= regrow(e, &D.gw_wflags, W0, W1, A);
  rc |= regrow(e, &D.gw_needs_ext, W0 * S::NXW, W1 * S::NXW, A);
  rc |= regrow(e, &D.gw_held, 0, 2 * W1, A);  // [2][W] scratch of a global stimulus
  rc |= regrow(e, &D.gw_needs_saved, W0 * S::NLW, W1 * S::NLW, A);
  int32_t Wp = 1;
  while ((size_t)Wp < W1) Wp <<= 1;
  if (Wp != D.Wp) {  // the round engine's tournament tree (rebuilt before use)
    rc |= regrow(e, &D.t_key, 0, 2 * (size_t)Wp, A);
    rc |= regrow(e, &D.t_idx, 0, 2 * (size_t)Wp, A);
  }
  const int32_t WB = (int32_t)((W1 + 63) / 64);
  if (WB != D.WB) rc |= restride(e, &D.holders, (size_t)D.N, (size_t)D.WB, (size_t)WB, e->graph_allocs);
  // [rounds][W] snapshots: a round's row holds the worker indices of its time (the SortedDict
  // rank then), padded with zeros to the current width -- the layout the reference-generated
  // fixtures record (tests/golden/gen_service.py, add_worker streams) -- so the new column is
  // appended, not inserted at `position`
  if (e->snap_rounds > 0) {
    const size_t R = (size_t)e->snap_rounds;
    rc |= restride(e, &D.snap_occ, R, W0, W1, A);
    rc |= restride(e, &D.snap_nbytes, R, W0, W1, A);
    rc |= restride(e, &D.snap_nproc, R, W0, W1, A);
    rc |= restride(e, &D.snap_flags, R, W0, W1, A);
  }
  if (rc) return rc;
  D.W = (int32_t)W1;
  D.WB = WB;
  D.Wp = Wp;
  const size_t pos = (size_t)position;
  if (pos < W0) {
    // Scheduler.workers is a SortedDict by address (:3746, inserted at :4353) and the canonical
    // worker order is its order: the new worker takes index pos, every later one moves up
    rc |= shift_rows(e, D.w_nthreads, W0, 1, pos);
    rc |= shift_rows(e, D.w_cap, W0, 1, pos);
    rc |= shift_rows(e, D.w_nproc, W0, 1, pos);
    rc |= shift_rows(e, D.w_plen, W0, 1, pos);
    rc |= shift_rows(e, D.w_pfx, W0, dgp::PMAX, pos);
    rc |= shift_rows(e, D.w_pcnt, W0, dgp::PMAX, pos);
    rc |= shift_rows(e, D.w_netocc, W0, 1, pos);
    rc |= shift_rows(e, D.w_nbytes, W0, 1, pos);
    rc |= shift_rows(e, D.w_flags, W0, 1, pos);
    rc |= shift_rows(e, D.w_itcslots, W0, 1, pos);
    rc |= shift_rows(e, D.w_lastcheck, W0, 1, pos);
    rc |= shift_rows(e, D.w_needs, W0, dgp::NEEDS_W, pos);
    rc |= shift_rows(e, D.gw_nproc, W0, 1, pos);
    rc |= shift_rows(e, D.gw_nthreads, W0, 1, pos);
    rc |= shift_rows(e, D.gw_cap, W0, 1, pos);
    rc |= shift_rows(e, D.gw_plen, W0, 1, pos);
    rc |= shift_rows(e, D.gw_pcnt, W0, S::PD, pos);
    rc |= shift_rows(e, D.gw_netocc, W0, 1, pos);
    rc |= shift_rows(e, D.gw_nbytes, W0, 1, pos);
    rc |= shift_rows(e, D.gw_mask, W0, 1, pos);
    rc |= shift_rows(e, D.gw_needs, W0, S::NLW, pos);
    rc |= shift_rows(e, D.gw_wflags, W0, 1, pos);
    rc |= shift_rows(e, D.gw_needs_ext, W0, S::NXW, pos);
    rc |= shift_rows(e, D.gw_needs_saved, W0, S::NLW, pos);
    if (rc) return rc;
    // worker indices held per task: holder_of, processing_on, the who_has bitsets
    hipLaunchKernelGGL(k_insert_worker_remap, dim3((unsigned)std::min<int64_t>((D.N + 255) / 256, 4096)), dim3(256), 0,
                       e->stream, D.holder_of, D.proc_on, D.holders, (int64_t)D.N, WB, (int32_t)pos);
    HIPCHK(e, hipGetLastError());
    {  // placements the stream engine has not sequenced carry their worker into holder_of at its start
      dgp::st::Pos ps;
      dgp::Ctl c0;
      HIPCHK(e, hipMemcpy(&ps, D.pos, sizeof ps, hipMemcpyDeviceToHost));
      if (int rc2 = read_ctl(e, &c0)) return rc2;
      const int64_t a = ps.runid_upto, b = (int64_t)c0.n_placed;
      if (b > a)
        hipLaunchKernelGGL(k_remap_range, dim3(64), dim3(256), 0, e->stream, D.pl_worker + a, b - a, (int32_t)pos);
      HIPCHK(e, hipGetLastError());
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    // the groups' last_worker and the restriction rows (valid workers stay ascending)
    auto remap_host = [&](int32_t* dptr, size_t n) -> int {
      if (!dptr || !n) return 0;
      std::vector<int32_t> h(n);
      HIPCHK(e, hipMemcpy(h.data(), dptr, n * 4, hipMemcpyDeviceToHost));
      for (auto& v : h) v += v >= (int32_t)pos ? 1 : 0;
      HIPCHK(e, hipMemcpy(dptr, h.data(), n * 4, hipMemcpyHostToDevice));
      return 0;
    };
    if (int rc2 = remap_host(D.g_lastw, (size_t)D.G)) return rc2;
    if (D.restr_ptr) {
      int64_t K = 0;
      HIPCHK(e, hipMemcpy(&K, D.restr_ptr + D.N, 8, hipMemcpyDeviceToHost));
      if (int rc2 = remap_host(const_cast<int32_t*>(D.restr_idx), (size_t)K)) return rc2;
    }
    if (D.restr_pool && e->rpool_used) {  // rows [len, workers...]: only the workers move
      std::vector<int32_t> h((size_t)e->rpool_used);
      HIPCHK(e, hipMemcpy(h.data(), D.restr_pool, h.size() * 4, hipMemcpyDeviceToHost));
      for (size_t q = 0; q < h.size();) {
        const int32_t len = h[q++];
        for (int32_t i = 0; i < len; i++, q++) h[q] += h[q] >= (int32_t)pos ? 1 : 0;
      }
      HIPCHK(e, hipMemcpy(const_cast<int32_t*>(D.restr_pool), h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
  }
  // the host mirrors follow only once every device step above succeeded
  e->paused_h.insert(e->paused_h.begin() + position, (uint8_t)(running ? 0 : 1));
  e->nthreads.insert(e->nthreads.begin() + pos, nthreads);
  D.total_nthreads += nthreads;
  const int32_t cap = D.sat_inf ? 0 : std::max((int32_t)std::ceil(D.saturation * nthreads), (int32_t)1);
  HIPCHK(e, hipMemcpy(D.w_nthreads + pos, &nthreads, 4, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_cap + pos, &cap, 4, hipMemcpyHostToDevice));
  // is_rootish (:2929-2947) reads total_nthreads: the groups' flags follow the new total
  {
    std::vector<uint8_t> tf = e->tflags_h;
    bool changed = false;
    for (int64_t t = 0; t < D.N; t++) {
      const int g = e->group_h[t];
      const bool gr = e->group_sizes[g] > D.total_nthreads * 2 && e->gdep_n[g] < 5 && e->gdep_len[g] < 5;
      const bool rs = !e->restr_h.empty() && (e->restr_h[t] & dgp::RF_RESTRICTED);
      const bool r = e->rootish_override_h[t] >= 0 ? e->rootish_override_h[t] != 0 : (gr && !rs);
      tf[t] = (uint8_t)((tf[t] & ~dgp::TF_ROOTISH) | (r ? dgp::TF_ROOTISH : 0));
      changed = changed || tf[t] != e->tflags_h[t];
    }
    if (changed) {
      HIPCHK(e, hipMemcpy(const_cast<uint8_t*>(D.tflags), tf.data(), D.N, hipMemcpyHostToDevice));
      e->tflags_h = tf;
    }
  }
  e->mode = 2;
  if (int rc2 = grow_logs(e, 0)) return rc2;
  if (int rc2 = sync_dev(e)) return rc2;
  if (!running) D.evf |= dgp::EVF_PAUSED;
  if (int rc2 = sync_dev(e)) return rc2;
  hipLaunchKernelGGL(dgp::st::k_add_worker, dim3(1), dim3(64), 0, e->stream, e->d_dev, e->d_aux + 3, (int32_t)pos,
                     running ? 1 : 0);
  HIPCHK(e, hipGetLastError());
  long long placed = 0;
  HIPCHK(e, hipMemcpyAsync(&placed, e->d_aux + 3, sizeof placed, hipMemcpyDeviceToHost, e->stream));
  dgp::Ctl c;
  if (int rc2 = check_device_error(e, &c)) return rc2;  // synchronises the stream
  if (n_new_placements) *n_new_placements = placed;
  e->last_placed = c.n_placed;
  return 0;
}

static int add_graph_impl(dgp_engine* e, int64_t n_new, const int64_t* dep_ptr, const int32_t* dep_idx,
                          const int64_t* prio, const int32_t* prefix_id, int32_t n_prefixes,
                          const double* prefix_default_duration, const int32_t* group_id, int32_t n_groups,
                          const uint8_t* wanted, const int8_t* rootish_override, int64_t* n_new_placements, bool defer);

int dgp_add_graph(dgp_engine* e, int64_t n_new, const int64_t* dep_ptr, const int32_t* dep_idx, const int64_t* prio,
                  const int32_t* prefix_id, int32_t n_prefixes, const double* prefix_default_duration,
                  const int32_t* group_id, int32_t n_groups, const uint8_t* wanted, const int8_t* rootish_override,
                  int64_t* n_new_placements) {
  return add_graph_impl(e, n_new, dep_ptr, dep_idx, prio, prefix_id, n_prefixes, prefix_default_duration, group_id,
                        n_groups, wanted, rootish_override, n_new_placements, false);
}

// (ABI 20) The task prefix table anew: the stream engine carries at most PX prefixes, a
// long-lived scheduler meets more over its session (TaskPrefix objects are per key_split
// name, scheduler.py:923-1031). The caller gives every task a slot in a table of
// n_prefixes live prefixes (the prefixes whose tasks are released / waiting / queued /
// processing / no-worker or in a worker's or the global task_prefix_count, :733-784,
// :1884-1903; a task of a prefix left out is in memory / erred / forgotten and its slot is
// never read) with each slot's default duration; the per-prefix state and every structure
// holding prefix ids (the workers' and the global dicts, the durations, the queue) then come
// from dgp_sync_workers / dgp_sync_globals (pending until dgp_sync_globals).
int dgp_remap_prefixes(dgp_engine* e, int32_t n_prefixes, const int32_t* task_prefix,
                       const double* prefix_default_duration) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (e->mode == 1) return fail(e, DGP_E_STATE, "engine advanced by a replay (dgp_run_rounds); dgp_reset first");
  if (e->posted) return fail(e, DGP_E_STATE, "a posted task-finished batch: dgp_tasks_finished_wait first");
  dgp::Dev& D = e->D;
  if (n_prefixes <= 0 || n_prefixes > dgp::st::PX || !task_prefix || !prefix_default_duration)
    return fail(e, DGP_E_ARG, "dgp_remap_prefixes: 1 .. 32 prefixes, every task's slot and each slot's default");
  for (int64_t t = 0; t < D.N; t++)
    if (task_prefix[t] < 0 || task_prefix[t] >= n_prefixes) return fail(e, DGP_E_ARG, "dgp_remap_prefixes: slot out of range");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  {  // no descriptor, duration row or record of the old numbering may be pending
    dgp::st::Pos ps;
    HIPCHK(e, hipMemcpy(&ps, D.pos, sizeof ps, hipMemcpyDeviceToHost));
    if (ps.pre > ps.seq || ps.walk != ps.rec_len)
      return fail(e, DGP_E_STATE, "dgp_remap_prefixes: the stream engine has prefetched stimuli or unfolded records");
  }
  if (n_prefixes > D.P) {  // per-prefix arrays one slot each (the round engine's table [N][P] too)
    int rc = 0;
    rc |= dalloc(e, &D.pdur_cur, n_prefixes, e->graph_allocs);
    rc |= dalloc(e, &D.pdur_walk, n_prefixes, e->graph_allocs);
    rc |= dalloc(e, &D.pdur_pre, n_prefixes, e->graph_allocs);
    rc |= dalloc(e, &D.pmaxexec, n_prefixes, e->graph_allocs);
    rc |= dalloc(e, &D.durv, (size_t)D.N * n_prefixes, e->graph_allocs);
    if (rc) return rc;
  }
  HIPCHK(e, hipMemcpy(const_cast<int32_t*>(D.prefix), task_prefix, (size_t)D.N * 4, hipMemcpyHostToDevice));
  e->h_prefix.assign(task_prefix, task_prefix + D.N);
  e->prefix_defaults.assign(prefix_default_duration, prefix_default_duration + n_prefixes);
  // placeholders until dgp_sync_globals brings each slot's TaskPrefix state
  std::vector<double> mx(n_prefixes, -1.0);
  for (double* p : {D.pdur_cur, D.pdur_walk, D.pdur_pre})
    HIPCHK(e, hipMemcpy(p, prefix_default_duration, (size_t)n_prefixes * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.pmaxexec, mx.data(), (size_t)n_prefixes * 8, hipMemcpyHostToDevice));
  D.P = n_prefixes;
  if (int rc = sync_dev(e)) return rc;
  e->pending_resync = true;  // the dicts hold the old numbering: dgp_sync_workers / _globals next
  e->mode = 2;
  return 0;
}

int dgp_set_priorities(dgp_engine* e, const int64_t* prio) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (e->mode == 1) return fail(e, DGP_E_STATE, "engine advanced by a replay (dgp_run_rounds); dgp_reset first");
  if (!prio) return fail(e, DGP_E_ARG, "dgp_set_priorities: prio missing");
  dgp::Dev& D = e->D;
  const int64_t N = D.N;
  const std::vector<int64_t>& dp = e->h_dep_ptr;
  const std::vector<int32_t>& di = e->h_dep_idx;
  std::vector<int32_t> order(N);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return prio[a] < prio[b]; });
  for (int64_t i = 1; i < N; i++)
    if (prio[order[i]] == prio[order[i - 1]]) return fail(e, DGP_E_ARG, "dgp_set_priorities: priorities must be unique");
  for (int64_t t = 0; t < N; t++)
    for (int64_t k = dp[t]; k < dp[t + 1]; k++)
      if (prio[di[k]] >= prio[t]) return fail(e, DGP_E_ARG, "dgp_set_priorities: priorities must be topological");
  // the dependents rows in the new order (the frontier order of _add_to_memory)
  const int64_t E = dp[N];
  std::vector<int64_t> dpt_ptr(N + 1, 0);
  for (int64_t k = 0; k < E; k++) dpt_ptr[di[k] + 1]++;
  for (int64_t t = 0; t < N; t++) dpt_ptr[t + 1] += dpt_ptr[t];
  std::vector<int32_t> dpt_idx(E > 0 ? E : 1);
  {
    std::vector<int64_t> fill(dpt_ptr.begin(), dpt_ptr.end() - 1);
    for (int64_t t = 0; t < N; t++)
      for (int64_t k = dp[t]; k < dp[t + 1]; k++) dpt_idx[fill[di[k]]++] = (int32_t)t;
    for (int64_t t = 0; t < N; t++)
      if (dpt_ptr[t + 1] - dpt_ptr[t] > 1)
        std::sort(dpt_idx.begin() + dpt_ptr[t], dpt_idx.begin() + dpt_ptr[t + 1],
                  [&](int32_t a, int32_t b) { return prio[a] < prio[b]; });
  }
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, hipMemcpy(const_cast<int64_t*>(D.prio), prio, (size_t)N * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(const_cast<int32_t*>(D.order), order.data(), (size_t)N * 4, hipMemcpyHostToDevice));
  if (E > 0) HIPCHK(e, hipMemcpy(const_cast<int32_t*>(D.dpt_idx), dpt_idx.data(), (size_t)E * 4, hipMemcpyHostToDevice));
  // the queue (qarr[qhead, qhead + qlen), ascending priority) re-sorted
  dgp::Ctl c;
  if (int rc = read_ctl(e, &c)) return rc;
  if (c.qlen > 1) {
    std::vector<int32_t> q((size_t)c.qlen);
    HIPCHK(e, hipMemcpy(q.data(), D.qarr + c.qhead, q.size() * 4, hipMemcpyDeviceToHost));
    std::stable_sort(q.begin(), q.end(), [&](int32_t a, int32_t b) { return prio[a] < prio[b]; });
    HIPCHK(e, hipMemcpy(D.qarr + c.qhead, q.data(), q.size() * 4, hipMemcpyHostToDevice));
  }
  e->h_prio.assign(prio, prio + N);
  return sync_dev(e);
}

int dgp_add_graph_deferred(dgp_engine* e, int64_t n_new, const int64_t* dep_ptr, const int32_t* dep_idx,
                           const int64_t* prio, const int32_t* prefix_id, int32_t n_prefixes,
                           const double* prefix_default_duration, const int32_t* group_id, int32_t n_groups,
                           const uint8_t* wanted, const int8_t* rootish_override) {
  return add_graph_impl(e, n_new, dep_ptr, dep_idx, prio, prefix_id, n_prefixes, prefix_default_duration, group_id,
                        n_groups, wanted, rootish_override, nullptr, true);
}

}  // extern "C"

namespace {
int stage_args(dgp_engine* e, std::initializer_list<std::pair<const void*, size_t>> parts, std::vector<char*>& out);
// is_rootish (:2929-2947) reads total_nthreads: the groups' flags follow a new total
int refresh_rootish(dgp_engine* e) {
  dgp::Dev& D = e->D;
  std::vector<uint8_t> tf = e->tflags_h;
  bool changed = false;
  for (int64_t t = 0; t < D.N; t++) {
    const int g = e->group_h[t];
    const bool gr = e->group_sizes[g] > D.total_nthreads * 2 && e->gdep_n[g] < 5 && e->gdep_len[g] < 5;
    const bool rs = !e->restr_h.empty() && (e->restr_h[t] & dgp::RF_RESTRICTED);
    const bool r = e->rootish_override_h[t] >= 0 ? e->rootish_override_h[t] != 0 : (gr && !rs);
    tf[t] = (uint8_t)((tf[t] & ~dgp::TF_ROOTISH) | (r ? dgp::TF_ROOTISH : 0));
    changed = changed || tf[t] != e->tflags_h[t];
  }
  if (changed) {
    HIPCHK(e, hipMemcpy(const_cast<uint8_t*>(D.tflags), tf.data(), D.N, hipMemcpyHostToDevice));
    e->tflags_h = tf;
  }
  return 0;
}
// every earlier task a new one depends on gains it as a waiter (_transition_released_waiting
// :2094-2099: dts.waiters.add(ts) for a dependency that is not released)
__global__ void k_add_waiters(int32_t* waiters, const int32_t* dep, const int32_t* cnt, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    waiters[dep[i]] += cnt[i];
}
// the later graph's tasks that are ready at once with dependencies (every one an earlier task
// in memory) go to decide_worker over their dependencies' holders: they become the frontier
// k_candidate_commbytes computes the candidates and comm bytes of
__global__ void k_ug_frontier(const dgp::Dev* __restrict__ Dp, int lo) {
  const dgp::Dev& D = *Dp;
  for (int64_t t = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < D.N; t += (int64_t)gridDim.x * blockDim.x)
    if (D.remaining[t] == 0 && D.dep_ptr[t + 1] > D.dep_ptr[t]) D.frontier[atomicAdd(&D.ctl->n_frontier, 1ull)] = (int)t;
}
__global__ void k_ug_frontier_reset(const dgp::Dev* __restrict__ Dp) {
  if (threadIdx.x == 0) {
    Dp->ctl->n_frontier = 0;
    Dp->ctl->pool_used = 0;
  }
}
}  // namespace

extern "C" {

static int graph_stimulus_impl(dgp_engine* e, bool ordered, int64_t n_order, const int32_t* order_task,
                               const int8_t* order_kind, const int64_t* order_ptr, const int32_t* order_idx,
                               int64_t* n_new_placements);
static int graph_stimulus_recompute(dgp_engine* e, int64_t n_order, const int32_t* order_task, const int8_t* order_kind,
                                    const int64_t* order_ptr, const int32_t* order_idx, int64_t* n_new_placements);

int dgp_graph_stimulus(dgp_engine* e, int64_t* n_new_placements) {
  return graph_stimulus_impl(e, false, 0, nullptr, nullptr, nullptr, nullptr, n_new_placements);
}

int dgp_graph_stimulus_ordered(dgp_engine* e, int64_t n_order, const int32_t* order_task, const int8_t* order_kind,
                               const int64_t* order_ptr, const int32_t* order_idx, int64_t* n_new_placements) {
  return graph_stimulus_impl(e, true, n_order, order_task, order_kind, order_ptr, order_idx, n_new_placements);
}

static int graph_stimulus_impl(dgp_engine* e, bool ordered, int64_t n_order, const int32_t* order_task,
                               const int8_t* order_kind, const int64_t* order_ptr, const int32_t* order_idx,
                               int64_t* n_new_placements) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (n_new_placements) *n_new_placements = 0;
  if (!e || !e->pending_resync || e->pending_lo < 0)
    return fail(e, DGP_E_STATE, "dgp_graph_stimulus: no appended graph (dgp_add_graph_deferred first)");
  dgp::Dev& D = e->D;
  const int64_t lo = e->pending_lo, N = D.N;
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  // the earlier tasks the new ones depend on: in memory (a replica), or waiting / queued /
  // processing (the new task waits on it); one released is recomputed (:2105-2106: the
  // recommendation machine with the scheduler's set orders, dgp_graph_stimulus_ordered); one
  // erred or forgotten would fail the new task (:4613-4618), which the engine leaves to the
  // scheduler
  std::vector<uint8_t> st((size_t)lo);
  HIPCHK(e, hipMemcpy(st.data(), D.state, (size_t)lo, hipMemcpyDeviceToHost));
  std::unordered_map<int32_t, int32_t> add;
  const std::vector<int64_t>& dp = e->h_dep_ptr;
  const std::vector<int32_t>& di = e->h_dep_idx;
  bool recompute = false;
  for (int64_t t = lo; t < N; t++)
    for (int64_t k = dp[t]; k < dp[t + 1]; k++) {
      const int32_t d = di[k];
      if (d >= lo) continue;
      const uint8_t sd = st[d];
      if (sd == dgp::S_ERRED || (e->tflags_h[d] & dgp::TF_FORGOTTEN) || (sd == dgp::S_RELEASED && !ordered))
        return fail(e, DGP_E_UNSUPPORTED, "dgp_graph_stimulus: an earlier dependency is released, erred or "
                                          "forgotten (recomputed by the scheduler): dgp_sync_* instead");
      recompute = recompute || sd == dgp::S_RELEASED;
      add[d] += 1;
    }
  if (recompute) return graph_stimulus_recompute(e, n_order, order_task, order_kind, order_ptr, order_idx,
                                                 n_new_placements);
  if (!add.empty()) {
    std::vector<int32_t> dd, cc;
    for (auto& kv : add) {
      dd.push_back(kv.first);
      cc.push_back(kv.second);
    }
    std::vector<char*> a;
    if (int rc = stage_args(e, {{dd.data(), dd.size() * 4}, {cc.data(), cc.size() * 4}}, a)) return rc;
    hipLaunchKernelGGL(k_add_waiters, dim3((unsigned)std::min<size_t>((dd.size() + 255) / 256, 1024)), dim3(256), 0,
                       e->stream, D.waiters, (const int32_t*)a[0], (const int32_t*)a[1], (int64_t)dd.size());
    HIPCHK(e, hipGetLastError());
  }
  e->pending_resync = false;
  e->pending_lo = -1;
  e->mode = 2;
  // the priority positions to scan: the new tasks follow every earlier one unless a user
  // priority outranks them (dgp_set_priorities re-ranked every task: scan them all)
  int64_t pmax_old = -1;
  for (int64_t t = 0; t < lo; t++) pmax_old = std::max(pmax_old, e->h_prio[t]);
  bool follows = true;
  for (int64_t t = lo; t < N && follows; t++) follows = e->h_prio[t] > pmax_old;
  if (int rc = grow_logs(e, 0)) return rc;
  if (int rc = sync_dev(e)) return rc;
  dgp::Ctl c0;
  if (int rc = read_ctl(e, &c0)) return rc;
  const dgp::Dev* DP = e->d_dev;
  hipStream_t s = e->stream;
  if (int rc = timed_launch(e, 3, [&] {
        launch_ug_init(e, lo);
        hipLaunchKernelGGL(k_ug_frontier_reset, dim3(1), dim3(64), 0, s, DP);
        hipLaunchKernelGGL(k_ug_frontier, dim3(grid_for(N - lo, 256, 2048)), dim3(256), 0, s, DP, (int)lo);
        hipLaunchKernelGGL(dgp::k_candidate_commbytes, dim3(grid_for(N - lo, 256, 2048)), dim3(256), 0, s, DP);
      }))
    return rc;
  if (int rc = launch_ug_dispatch(e, follows ? (int)lo : 0, (int)lo)) return rc;
  if (int rc = set_runids(e)) return rc;
  dgp::Ctl c;
  if (int rc = check_device_error(e, &c)) return rc;
  if (!follows && c.qlen > 1) {  // the queue (HeapSet by priority) with the new root-ish tasks in their place
    std::vector<int32_t> q((size_t)c.qlen);
    HIPCHK(e, hipMemcpy(q.data(), D.qarr + c.qhead, q.size() * 4, hipMemcpyDeviceToHost));
    std::stable_sort(q.begin(), q.end(), [&](int32_t a, int32_t b) { return e->h_prio[a] < e->h_prio[b]; });
    HIPCHK(e, hipMemcpy(D.qarr + c.qhead, q.data(), q.size() * 4, hipMemcpyHostToDevice));
  }
  if (n_new_placements) *n_new_placements = (int64_t)(c.n_placed - c0.n_placed);
  e->last_placed = c.n_placed;
  return 0;
}

static int add_graph_impl(dgp_engine* e, int64_t n_new, const int64_t* dep_ptr, const int32_t* dep_idx,
                          const int64_t* prio, const int32_t* prefix_id, int32_t n_prefixes,
                          const double* prefix_default_duration, const int32_t* group_id, int32_t n_groups,
                          const uint8_t* wanted, const int8_t* rootish_override, int64_t* n_new_placements, bool defer) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (n_new_placements) *n_new_placements = 0;
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (e->mode == 1) return fail(e, DGP_E_STATE, "engine advanced by a replay (dgp_run_rounds); dgp_reset first");
  if (e->pending_resync) return fail(e, DGP_E_STATE, "dgp_add_graph: dgp_sync_* first (a later graph depends on earlier tasks)");
  dgp::Dev& D = e->D;
  if (std::count_if(e->paused_h.begin(), e->paused_h.end(), [](uint8_t v) { return v != 0; }))
    return fail(e, DGP_E_STATE, "dgp_add_graph: not while a worker is paused or removed");
  if (n_new <= 0 || !dep_ptr || !prio || !prefix_id || !prefix_default_duration || !group_id || !wanted ||
      !rootish_override)
    return fail(e, DGP_E_ARG, "dgp_add_graph: bad arguments");
  const int64_t N0 = D.N, E0 = e->E, N1 = N0 + n_new;
  const int32_t P0 = D.P, G0 = D.G;
  if (n_prefixes < P0 || n_groups < G0) return fail(e, DGP_E_ARG, "dgp_add_graph: prefix / group tables shrank");
  if (n_prefixes > dgp::st::PX)
    return fail(e, DGP_E_STATE, "dgp_add_graph: more task prefixes than the stream engine carries (32)");
  if (dep_ptr[0] != 0) return fail(e, DGP_E_ARG, "dgp_add_graph: bad dep_ptr");
  for (int64_t t = 0; t < n_new; t++)
    if (dep_ptr[t + 1] < dep_ptr[t]) return fail(e, DGP_E_ARG, "dgp_add_graph: dep_ptr not monotone");
  const int64_t En = dep_ptr[n_new];
  if (En > 0 && !dep_idx) return fail(e, DGP_E_ARG, "dgp_add_graph: dep_idx missing");
  // a dependency is a task of the new graph (0 .. n_new-1) or an earlier task t (-1 - t)
  bool ext_deps = false;
  for (int64_t k = 0; k < En; k++) {
    if (dep_idx[k] >= n_new || (dep_idx[k] < 0 && -1 - (int64_t)dep_idx[k] >= N0))
      return fail(e, DGP_E_ARG, "dgp_add_graph: dependency out of range");
    ext_deps = ext_deps || dep_idx[k] < 0;
  }
  const int64_t pmax = *std::max_element(e->h_prio.begin(), e->h_prio.end());
  for (int64_t t = 0; t < n_new; t++)
    if (prio[t] <= pmax) return fail(e, DGP_E_ARG, "dgp_add_graph: new priorities must follow every earlier task's");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  // the whole graph, old tasks first
  std::vector<int64_t> dp(e->h_dep_ptr), pr(e->h_prio);
  std::vector<int32_t> di(e->h_dep_idx), pf(e->h_prefix), gr(e->group_h);
  std::vector<uint8_t> wa(e->h_wanted);
  std::vector<int8_t> ov(e->rootish_override_h);
  for (int64_t t = 0; t < n_new; t++) {
    dp.push_back(E0 + dep_ptr[t + 1]);
    pr.push_back(prio[t]);
    pf.push_back(prefix_id[t]);
    gr.push_back(group_id[t]);
    wa.push_back(wanted[t]);
    ov.push_back(rootish_override[t]);
  }
  for (int64_t t = 0; t < n_new; t++) {  // rows ascending in the whole graph's numbering
    const size_t r0 = di.size();
    for (int64_t k = dep_ptr[t]; k < dep_ptr[t + 1]; k++)
      di.push_back(dep_idx[k] >= 0 ? (int32_t)(dep_idx[k] + N0) : (int32_t)(-1 - (int64_t)dep_idx[k]));
    std::sort(di.begin() + r0, di.end());
  }
  std::vector<double> pd(e->prefix_defaults);
  pd.resize(n_prefixes);
  for (int32_t q = P0; q < n_prefixes; q++) pd[q] = prefix_default_duration[q];
  // released + waiting per group after the new tasks arrive (they start released)
  std::vector<int64_t> relwait(n_groups, 0);
  HIPCHK(e, hipMemcpy(relwait.data(), D.g_relwait, (size_t)G0 * 8, hipMemcpyDeviceToHost));
  for (int64_t t = 0; t < n_new; t++) relwait[group_id[t]]++;
  const dgp::Dev old = D;
  const std::vector<uint8_t> old_tf = e->tflags_h, old_restr = e->restr_h;
  const int64_t old_rpool_used = e->rpool_used, old_rpool_cap = e->rpool_cap;
  const int64_t old_rlog = D.rlog_cap;
  e->log_min[0] = D.pl_cap + n_new;
  e->log_min[1] = D.sv_cap + n_new;
  e->log_min[2] = D.rlog_cap + 2 * n_new;
  std::vector<void*> old_allocs;
  old_allocs.swap(e->graph_allocs);
  e->have_graph = false;
  if (int rc = upload_graph(e, N1, dp.data(), di.data(), pr.data(), pf.data(), n_prefixes, pd.data(), gr.data(),
                            n_groups, wa.data(), ov.data())) {
    free_list(e->graph_allocs);  // the engine keeps its old graph
    e->graph_allocs.swap(old_allocs);
    D = old;
    return rc;
  }
  e->have_graph = true;
  // the dynamic state of the old tasks carried over; the new ones as dgp_reset leaves them
  hipStream_t s = e->stream;
  auto carry = [&](void* dst, const void* src, size_t old_bytes, size_t new_bytes, int fill) -> hipError_t {
    hipError_t st = hipMemsetAsync(dst, fill, new_bytes, s);
    if (st == hipSuccess && old_bytes) st = hipMemcpyAsync(dst, src, old_bytes, hipMemcpyDeviceToDevice, s);
    return st;
  };
  const size_t n0 = N0, n1 = N1;
  HIPCHK(e, carry(D.res_nbytes, old.res_nbytes, n0 * 8, n1 * 8, 0xff));
  HIPCHK(e, carry(D.res_start, old.res_start, n0 * 8, n1 * 8, 0));
  HIPCHK(e, carry(D.res_stop, old.res_stop, n0 * 8, n1 * 8, 0));
  HIPCHK(e, carry(D.state, old.state, n0, n1, 0));
  HIPCHK(e, carry(D.remaining, old.remaining, n0 * 4, n1 * 4, 0));
  HIPCHK(e, carry(D.waiters, old.waiters, n0 * 4, n1 * 4, 0));
  HIPCHK(e, carry(D.proc_on, old.proc_on, n0 * 4, n1 * 4, 0xff));
  HIPCHK(e, carry(D.cur_nbytes, old.cur_nbytes, n0 * 8, n1 * 8, 0xff));
  HIPCHK(e, carry(D.holders, old.holders, n0 * D.WB * 8, n1 * D.WB * 8, 0));
  HIPCHK(e, carry(D.ready_key, old.ready_key, n0 * 8, n1 * 8, 0));
  HIPCHK(e, carry(D.release_key, old.release_key, n0 * 8, n1 * 8, 0));
  HIPCHK(e, carry(D.cand_n, old.cand_n, n0 * 4, n1 * 4, 0));
  HIPCHK(e, carry(D.qarr, old.qarr, n0 * 4, n1 * 4, 0));
  const size_t p0 = old.pl_cap, p1 = D.pl_cap;
  HIPCHK(e, carry(D.pl_task, old.pl_task, p0 * 4, p1 * 4, 0));
  HIPCHK(e, carry(D.pl_worker, old.pl_worker, p0 * 4, p1 * 4, 0));
  HIPCHK(e, carry(D.pl_comm, old.pl_comm, p0 * 8, p1 * 8, 0));
  HIPCHK(e, carry(D.pl_start, old.pl_start, p0 * 8, p1 * 8, 0));
  HIPCHK(e, carry(D.pl_wsnbytes, old.pl_wsnbytes, p0 * 8, p1 * 8, 0));
  HIPCHK(e, carry(D.pl_route, old.pl_route, p0, p1, 0));
  HIPCHK(e, carry(D.run_id, old.run_id, n0 * 4, n1 * 4, 0xff));
  HIPCHK(e, carry(D.holder_of, old.holder_of, n0 * 4, n1 * 4, 0xff));
  HIPCHK(e, carry(D.tdyn, old.tdyn, n0, n1, 0));
  HIPCHK(e, carry(D.fr_mark, old.fr_mark, n0 * 4, n1 * 4, 0xff));
  HIPCHK(e, carry(D.rel_mark, old.rel_mark, n0 * 4, n1 * 4, 0xff));
  HIPCHK(e, carry(D.rlog, old.rlog, (size_t)old_rlog * sizeof(dgp::st::SRec), (size_t)D.rlog_cap * sizeof(dgp::st::SRec), 0));
  HIPCHK(e, carry(D.sv_task, old.sv_task, (size_t)old.sv_cap * 4, (size_t)D.sv_cap * 4, 0));
  HIPCHK(e, carry(D.sv_worker, old.sv_worker, (size_t)old.sv_cap * 4, (size_t)D.sv_cap * 4, 0));
  HIPCHK(e, carry(D.sv_cseq, old.sv_cseq, n0 * 4, n1 * 4, 0xff));
  HIPCHK(e, carry(D.svc_len, old.svc_len, 8, 8, 0));
  // prefixes: TaskPrefix state of the known ones kept, the new ones at their defaults
  for (double* const* pp : {&D.pdur_cur, &D.pdur_walk, &D.pdur_pre}) {
    HIPCHK(e, hipMemcpyAsync(*pp, pd.data(), (size_t)n_prefixes * 8, hipMemcpyHostToDevice, s));
  }
  HIPCHK(e, hipMemcpyAsync(D.pdur_cur, old.pdur_cur, (size_t)P0 * 8, hipMemcpyDeviceToDevice, s));
  HIPCHK(e, hipMemcpyAsync(D.pdur_walk, old.pdur_walk, (size_t)P0 * 8, hipMemcpyDeviceToDevice, s));
  HIPCHK(e, hipMemcpyAsync(D.pdur_pre, old.pdur_pre, (size_t)P0 * 8, hipMemcpyDeviceToDevice, s));
  HIPCHK(e, carry(D.pmaxexec, old.pmaxexec, (size_t)P0 * 8, (size_t)n_prefixes * 8, 0));
  if (n_prefixes > P0) {  // the new prefixes: no max_exec_time yet (the known ones keep theirs)
    std::vector<double> mx(n_prefixes - P0, -1.0);
    HIPCHK(e, hipMemcpyAsync(D.pmaxexec + P0, mx.data(), mx.size() * 8, hipMemcpyHostToDevice, s));
  }
  // groups
  HIPCHK(e, hipMemcpyAsync(D.g_relwait, relwait.data(), (size_t)n_groups * 8, hipMemcpyHostToDevice, s));
  HIPCHK(e, carry(D.g_left, old.g_left, (size_t)G0 * 8, (size_t)n_groups * 8, 0));
  HIPCHK(e, carry(D.g_lastw, old.g_lastw, (size_t)G0 * 4, (size_t)n_groups * 4, 0xff));
  HIPCHK(e, hipStreamSynchronize(s));
  // task flags the graph upload does not know: forgotten rows (resync) and restrictions
  for (int64_t t = 0; t < N0; t++) e->tflags_h[t] |= (uint8_t)(old_tf[t] & dgp::TF_FORGOTTEN);
  if (old.restr_ovr) {  // rows changed after the upload: the overrides and their pool carried over
    int64_t* ov = nullptr;
    int32_t* pl = nullptr;
    if (dalloc(e, &ov, N1, e->graph_allocs) || dalloc(e, &pl, std::max<int64_t>(old_rpool_cap, 1), e->graph_allocs))
      return DGP_E_HIP;
    HIPCHK(e, carry(ov, old.restr_ovr, (size_t)N0 * 8, (size_t)N1 * 8, 0xff));
    if (old_rpool_used)
      HIPCHK(e, hipMemcpyAsync(pl, old.restr_pool, (size_t)old_rpool_used * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(e, hipStreamSynchronize(s));
    D.restr_ovr = ov;
    D.restr_pool = pl;
    e->rpool_used = old_rpool_used;
    e->rpool_cap = std::max<int64_t>(old_rpool_cap, 1);
  }
  if (old.restr_flags) {  // the earlier tasks keep their restrictions; the new ones have none
    std::vector<int64_t> rp(N1 + 1);
    HIPCHK(e, hipMemcpy(rp.data(), old.restr_ptr, (N0 + 1) * 8, hipMemcpyDeviceToHost));
    const int64_t K = rp[N0];
    for (int64_t t = N0; t < N1; t++) rp[t + 1] = K;
    std::vector<int32_t> ri(std::max<int64_t>(K, 1), 0);
    if (K) HIPCHK(e, hipMemcpy(ri.data(), old.restr_idx, K * 4, hipMemcpyDeviceToHost));
    e->restr_h = old_restr;
    e->restr_h.resize(N1, 0);
    int64_t* rpd = nullptr;
    int32_t* rid = nullptr;
    uint8_t* rfd = nullptr;
    int rc = 0;
    rc |= dalloc(e, &rpd, N1 + 1, e->graph_allocs);
    rc |= dalloc(e, &rid, (int64_t)ri.size(), e->graph_allocs);
    rc |= dalloc(e, &rfd, N1, e->graph_allocs);
    if (rc) return DGP_E_HIP;
    HIPCHK(e, hipMemcpy(rpd, rp.data(), (N1 + 1) * 8, hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(rid, ri.data(), ri.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(rfd, e->restr_h.data(), N1, hipMemcpyHostToDevice));
    D.restr_ptr = rpd;
    D.restr_idx = rid;
    D.restr_flags = rfd;
    // a restricted task is not root-ish unless _rootish says so (is_rootish :2929-2947)
    for (int64_t t = 0; t < N0; t++)
      if ((e->restr_h[t] & dgp::RF_RESTRICTED) && e->rootish_override_h[t] < 0)
        e->tflags_h[t] &= (uint8_t)~dgp::TF_ROOTISH;
  }
  HIPCHK(e, hipMemcpy(const_cast<uint8_t*>(D.tflags), e->tflags_h.data(), N1, hipMemcpyHostToDevice));
  free_list(old_allocs);
  if (ext_deps || defer) {
    // the new tasks stay released: the scheduler decides this update_graph stimulus itself
    // (the new tasks' waiting_on / the earlier tasks' waiters, any placement it makes) and
    // the caller hands over its state (dgp_sync_*) before the next stimulus
    e->pending_resync = true;
    e->pending_lo = N0;
    e->mode = 2;
    if (int rc = sync_dev(e)) return rc;
    return 0;
  }
  // the update_graph stimulus of the new tasks (:4600-4651): released -> waiting, the
  // runnable ones (no dependency: the new graph is independent of the old) to processing
  // or queued in priority order
  if (int rc = sync_dev(e)) return rc;
  dgp::Ctl c0;
  if (int rc = read_ctl(e, &c0)) return rc;
  const dgp::Dev* DP = e->d_dev;
  if (int rc = timed_launch(e, 3, [&] {
        launch_ug_init(e, N0);
      }))
    return rc;
  if (int rc = launch_ug_dispatch(e, (int)N0, (int)N0)) return rc;
  if (int rc = set_runids(e)) return rc;
  e->mode = 2;
  dgp::Ctl c;
  if (int rc = check_device_error(e, &c)) return rc;
  if (n_new_placements) *n_new_placements = (int64_t)(c.n_placed - c0.n_placed);
  e->last_placed = c.n_placed;
  return 0;
}

}  // extern "C"

namespace {

// the common preconditions of a service event: the stream engine in service mode
int event_ready(dgp_engine* e, const char* what) {
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (e->pending_resync && strncmp(what, "dgp_sync_", 9) != 0 && strcmp(what, "dgp_remove_worker") != 0)
    return fail(e, DGP_E_STATE, std::string(what) + ": the scheduler decides the stimulus of a graph that depends on "
                                                    "earlier tasks; dgp_sync_* first");
  if (e->mode == 1) return fail(e, DGP_E_STATE, "engine advanced by a replay (dgp_run_rounds); dgp_reset first");
  if (!(e->D.P <= dgp::st::PX))
    return fail(e, DGP_E_STATE, std::string(what) + ": the round-kernel engine (more than 32 prefixes) has no "
                                                    "service events");
  HIPCHK(e, hipSetDevice(e->device));
  e->mode = 2;
  return 0;
}

// copy the event's argument arrays (each padded to 16 bytes) into the device staging
int stage_args(dgp_engine* e, std::initializer_list<std::pair<const void*, size_t>> parts, std::vector<char*>& out) {
  size_t need = 0;
  for (auto& p : parts) need += (p.second + 15) & ~(size_t)15;
  if (need > e->d_ev_cap) {
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->d_ev) (void)hipFree(e->d_ev);
    e->d_ev = nullptr;
    e->d_ev_cap = 0;
    const size_t cap = std::max<size_t>(need, 4096);
    HIPCHK(e, hipMalloc((void**)&e->d_ev, cap));
    e->d_ev_cap = cap;
  }
  size_t off = 0;
  out.clear();
  for (auto& p : parts) {
    out.push_back(e->d_ev + off);
    if (p.second) HIPCHK(e, hipMemcpyAsync(e->d_ev + off, p.first, p.second, hipMemcpyHostToDevice, e->stream));
    off += (p.second + 15) & ~(size_t)15;
  }
  return 0;
}

// a one-wave event kernel that may refill the queue: run it, report its placements
template <class F>
int event_with_refill(dgp_engine* e, F&& launch, int64_t* n_new_placements) {
  if (int rc = grow_logs(e, 0)) return rc;
  if (int rc = sync_dev(e)) return rc;
  launch();
  HIPCHK(e, hipGetLastError());
  long long placed = 0;
  HIPCHK(e, hipMemcpyAsync(&placed, e->d_aux + 3, sizeof placed, hipMemcpyDeviceToHost, e->stream));
  dgp::Ctl c;
  if (int rc = check_device_error(e, &c)) return rc;  // synchronises the stream
  if (n_new_placements) *n_new_placements = placed;
  e->last_placed = c.n_placed;
  return 0;
}

}  // namespace

extern "C" {

int dgp_add_replicas(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (int rc = event_ready(e, "dgp_add_replicas")) return rc;
  if (n < 0 || (n > 0 && (!task || !worker))) return fail(e, DGP_E_ARG, "dgp_add_replicas: bad batch");
  for (int64_t i = 0; i < n; i++)
    if (task[i] < 0 || task[i] >= e->D.N || worker[i] < 0 || worker[i] >= e->D.W)
      return fail(e, DGP_E_ARG, "dgp_add_replicas: task or worker out of range");
  if (n == 0) return 0;
  std::vector<char*> a;
  if (int rc = stage_args(e, {{task, n * 4}, {worker, n * 4}}, a)) return rc;
  e->D.evf |= dgp::EVF_MULTI;
  if (int rc = sync_dev(e)) return rc;
  hipLaunchKernelGGL(dgp::ev::k_ev_add_replicas, dim3(1), dim3(64), 0, e->stream, e->d_dev, (const int32_t*)a[0],
                     (const int32_t*)a[1], (int)n);
  HIPCHK(e, hipGetLastError());
  return check_device_error(e);
}

int dgp_remove_replicas(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (int rc = event_ready(e, "dgp_remove_replicas")) return rc;
  if (n < 0 || (n > 0 && (!task || !worker))) return fail(e, DGP_E_ARG, "dgp_remove_replicas: bad batch");
  for (int64_t i = 0; i < n; i++)
    if (task[i] < 0 || task[i] >= e->D.N || worker[i] < 0 || worker[i] >= e->D.W)
      return fail(e, DGP_E_ARG, "dgp_remove_replicas: task or worker out of range");
  if (n == 0) return 0;
  std::vector<char*> a;
  if (int rc = stage_args(e, {{task, n * 4}, {worker, n * 4}}, a)) return rc;
  e->D.evf |= dgp::EVF_MULTI;
  if (int rc = sync_dev(e)) return rc;
  hipLaunchKernelGGL(dgp::ev::k_ev_remove_replicas, dim3(1), dim3(64), 0, e->stream, e->d_dev, (const int32_t*)a[0],
                     (const int32_t*)a[1], (int)n);
  HIPCHK(e, hipGetLastError());
  return check_device_error(e);
}

int dgp_set_worker_status(dgp_engine* e, int32_t worker, int32_t running, int64_t* n_new_placements) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (n_new_placements) *n_new_placements = 0;
  if (int rc = event_ready(e, "dgp_set_worker_status")) return rc;
  if (worker < 0 || worker >= e->D.W) return fail(e, DGP_E_ARG, "dgp_set_worker_status: worker out of range");
  const uint8_t paused = running ? 0 : 1;
  if (e->paused_h[worker] == 2) return fail(e, DGP_E_ARG, "dgp_set_worker_status: the worker was removed");
  if (e->paused_h[worker] == paused) return 0;  // ws.status == prev_status: nothing (:5858-5859)
  e->paused_h[worker] = paused;
  e->D.evf |= dgp::EVF_PAUSED;
  return event_with_refill(e, [&] {
    hipLaunchKernelGGL(dgp::ev::k_ev_worker_status, dim3(1), dim3(64), 0, e->stream, e->d_dev, worker,
                       running ? 1 : 0, e->d_aux + 3);
  }, n_new_placements);
}

int dgp_long_running(dgp_engine* e, int32_t task, double compute_duration, int64_t* n_new_placements) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (n_new_placements) *n_new_placements = 0;
  if (int rc = event_ready(e, "dgp_long_running")) return rc;
  if (task < 0 || task >= e->D.N) return fail(e, DGP_E_ARG, "dgp_long_running: task out of range");
  e->D.evf |= dgp::EVF_LR;
  return event_with_refill(e, [&] {
    hipLaunchKernelGGL(dgp::ev::k_ev_long_running, dim3(1), dim3(64), 0, e->stream, e->d_dev, task,
                       compute_duration, e->d_aux + 3);
  }, n_new_placements);
}

int dgp_release_tasks(dgp_engine* e, int64_t n, const int32_t* task, const uint8_t* forget, int64_t* n_new_placements) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (n_new_placements) *n_new_placements = 0;
  if (int rc = event_ready(e, "dgp_release_tasks")) return rc;
  dgp::Dev& D = e->D;
  if (n < 0 || (n > 0 && (!task || !forget))) return fail(e, DGP_E_ARG, "dgp_release_tasks: bad batch");
  for (int64_t i = 0; i < n; i++)
    if (task[i] < 0 || task[i] >= D.N) return fail(e, DGP_E_ARG, "dgp_release_tasks: task out of range");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  // results in memory, released tasks and cancelled work (waiting, processing, queued,
  // no-worker); an erred or forgotten task is the scheduler's (then dgp_sync_*)
  std::vector<uint8_t> st((size_t)D.N);
  HIPCHK(e, hipMemcpy(st.data(), D.state, (size_t)D.N, hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < n; i++) {
    const uint8_t x = st[task[i]];
    if (x > dgp::S_MEMORY || (e->tflags_h[task[i]] & dgp::TF_FORGOTTEN))
      return fail(e, DGP_E_UNSUPPORTED, "dgp_release_tasks: an erred or forgotten task (the scheduler decides, "
                                        "then dgp_sync_*)");
  }
  // who_wants emptied; forgotten ones leave SchedulerState.tasks (their rows stay, flagged)
  for (int64_t i = 0; i < n; i++) {
    const int32_t t = task[i];
    e->tflags_h[t] = (uint8_t)((e->tflags_h[t] & ~dgp::TF_WANTED) | (forget[i] ? dgp::TF_FORGOTTEN : 0));
    e->h_wanted[t] = 0;
  }
  HIPCHK(e, hipMemcpy(const_cast<uint8_t*>(D.tflags), e->tflags_h.data(), D.N, hipMemcpyHostToDevice));
  std::vector<char*> a;
  if (int rc = stage_args(e, {{task, (size_t)n * 4}}, a)) return rc;
  return event_with_refill(e, [&] {
    hipLaunchKernelGGL(dgp::ev::k_ev_release_tasks, dim3(1), dim3(64), 0, e->stream, e->d_dev, (const int32_t*)a[0],
                       (int)n, e->d_aux + 3);
  }, n_new_placements);
}

int dgp_heartbeat(dgp_engine* e, double bandwidth, int64_t n, const int32_t* prefix, const double* duration) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (int rc = event_ready(e, "dgp_heartbeat")) return rc;
  if (!(bandwidth > 0) || n < 0 || (n > 0 && (!prefix || !duration)))
    return fail(e, DGP_E_ARG, "dgp_heartbeat: bandwidth must be > 0; prefixes and durations");
  for (int64_t i = 0; i < n; i++)
    if (prefix[i] < 0 || prefix[i] >= e->D.P) return fail(e, DGP_E_ARG, "dgp_heartbeat: prefix out of range");
  e->D.bandwidth = bandwidth;
  if (n > 0) {
    std::vector<char*> a;
    if (int rc = stage_args(e, {{prefix, n * 4}, {duration, n * 8}}, a)) return rc;
    if (int rc = sync_dev(e)) return rc;
    hipLaunchKernelGGL(dgp::ev::k_ev_heartbeat, dim3(1), dim3(64), 0, e->stream, e->d_dev, (const int32_t*)a[0],
                       (const double*)a[1], (int)n);
    HIPCHK(e, hipGetLastError());
  }
  if (int rc = sync_dev(e)) return rc;
  return check_device_error(e);
}

int dgp_set_worker_flags(dgp_engine* e, int64_t n, const int32_t* worker, const uint8_t* idle, const uint8_t* saturated) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (int rc = event_ready(e, "dgp_set_worker_flags")) return rc;
  if (n < 0 || (n > 0 && (!worker || !idle || !saturated))) return fail(e, DGP_E_ARG, "dgp_set_worker_flags: bad batch");
  for (int64_t i = 0; i < n; i++) {
    if (worker[i] < 0 || worker[i] >= e->D.W) return fail(e, DGP_E_ARG, "dgp_set_worker_flags: worker out of range");
    if (e->paused_h[worker[i]] && (idle[i] || saturated[i]))
      return fail(e, DGP_E_ARG, "dgp_set_worker_flags: a paused worker is neither idle nor saturated");
  }
  if (n == 0) return 0;
  std::vector<char*> a;
  if (int rc = stage_args(e, {{worker, n * 4}, {idle, (size_t)n}, {saturated, (size_t)n}}, a)) return rc;
  if (int rc = sync_dev(e)) return rc;
  hipLaunchKernelGGL(dgp::ev::k_ev_worker_flags, dim3(1), dim3(64), 0, e->stream, e->d_dev, (const int32_t*)a[0],
                     (const uint8_t*)a[1], (const uint8_t*)a[2], (int)n);
  HIPCHK(e, hipGetLastError());
  return check_device_error(e);
}

int dgp_set_wanted(dgp_engine* e, int64_t n, const int32_t* task, const uint8_t* wanted) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (int rc = event_ready(e, "dgp_set_wanted")) return rc;
  if (n < 0 || (n > 0 && (!task || !wanted))) return fail(e, DGP_E_ARG, "dgp_set_wanted: bad batch");
  for (int64_t i = 0; i < n; i++)
    if (task[i] < 0 || task[i] >= e->D.N) return fail(e, DGP_E_ARG, "dgp_set_wanted: task out of range");
  if (n == 0) return 0;
  HIPCHK(e, hipStreamSynchronize(e->stream));
  std::vector<uint8_t>& tf = e->tflags_h;
  for (int64_t i = 0; i < n; i++) {
    const int32_t t = task[i];
    tf[t] = (uint8_t)((tf[t] & ~dgp::TF_WANTED) | (wanted[i] ? dgp::TF_WANTED : 0));
    e->h_wanted[t] = wanted[i] ? 1 : 0;
    HIPCHK(e, hipMemcpy(const_cast<uint8_t*>(e->D.tflags) + t, &tf[t], 1, hipMemcpyHostToDevice));
  }
  return 0;
}

int dgp_task_erred(dgp_engine* e, int32_t task, int64_t* n_new_placements) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (n_new_placements) *n_new_placements = 0;
  if (int rc = event_ready(e, "dgp_task_erred")) return rc;
  if (task < 0 || task >= e->D.N) return fail(e, DGP_E_ARG, "dgp_task_erred: task out of range");
  return event_with_refill(e, [&] {
    hipLaunchKernelGGL(dgp::ev::k_ev_task_erred, dim3(1), dim3(64), 0, e->stream, e->d_dev, task, e->d_aux + 3);
  }, n_new_placements);
}

int dgp_remove_worker(dgp_engine* e, int32_t worker) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (int rc = event_ready(e, "dgp_remove_worker")) return rc;
  if (worker < 0 || worker >= e->D.W) return fail(e, DGP_E_ARG, "dgp_remove_worker: worker out of range");
  if (e->paused_h[worker] == 2) return 0;  // already removed ("already-removed" :5196-5197)
  HIPCHK(e, hipStreamSynchronize(e->stream));
  // Scheduler.remove_worker's worker table part (:5213-5231): the WorkerState leaves workers,
  // running, idle, idle_task_count and saturated and total_nthreads; its index stays (the
  // canonical order of the others is unchanged) as a worker that is never a candidate
  int64_t placed = 0;
  if (!e->paused_h[worker])
    if (int rc = dgp_set_worker_status(e, worker, 0, &placed)) return rc;
  e->paused_h[worker] = 2;
  e->D.total_nthreads -= e->nthreads[worker];
  return refresh_rootish(e);
}

// the order rows of dgp_lose_worker_ordered / dgp_graph_stimulus_ordered: sorted by (task,
// kind); kind 0 a permutation of the task's dependencies, kinds 1 / 2 distinct dependents
static int check_order_rows(dgp_engine* e, int64_t n_order, const int32_t* order_task, const int8_t* order_kind,
                            const int64_t* order_ptr, const int32_t* order_idx, const char* what) {
  const dgp::Dev& D = e->D;
  if (n_order < 0 || n_order > 2 * D.N || (n_order && (!order_task || !order_kind || !order_ptr || !order_idx)))
    return fail(e, DGP_E_ARG, std::string(what) + ": bad order rows");
  if (n_order && order_ptr[0] != 0) return fail(e, DGP_E_ARG, std::string(what) + ": order_ptr[0] != 0");
  const std::vector<int64_t>& dp = e->h_dep_ptr;
  const std::vector<int32_t>& di = e->h_dep_idx;
  for (int64_t i = 0; i < n_order; i++) {
    const int32_t t = order_task[i];
    const int k = order_kind[i];
    if (t < 0 || t >= D.N || k < dgp::ev::LO_DEPS || k > dgp::ev::LO_DEPENDENTS || order_ptr[i + 1] < order_ptr[i])
      return fail(e, DGP_E_ARG, std::string(what) + ": bad order row");
    if (i > 0 && (order_task[i - 1] > t || (order_task[i - 1] == t && order_kind[i - 1] >= k)))
      return fail(e, DGP_E_ARG, std::string(what) + ": order rows not sorted by (task, kind)");
    std::vector<int32_t> r(order_idx + order_ptr[i], order_idx + order_ptr[i + 1]);
    for (int32_t x : r)
      if (x < 0 || x >= D.N) return fail(e, DGP_E_ARG, std::string(what) + ": task out of range");
    std::sort(r.begin(), r.end());
    if (std::adjacent_find(r.begin(), r.end()) != r.end())
      return fail(e, DGP_E_ARG, std::string(what) + ": a task twice in one row");
    if (k == dgp::ev::LO_DEPS) {
      std::vector<int32_t> own(di.begin() + dp[t], di.begin() + dp[t + 1]);
      std::sort(own.begin(), own.end());
      if (own != r) return fail(e, DGP_E_ARG, std::string(what) + ": a dependency row is not the task's dependencies");
    } else {
      for (int32_t y : r)
        if (std::find(di.begin() + dp[y], di.begin() + dp[y + 1], t) == di.begin() + dp[y + 1])
          return fail(e, DGP_E_ARG, std::string(what) + ": a waiters / dependents row names a task that does not depend on it");
    }
  }
  return 0;
}

// a later graph's update_graph stimulus that recomputes released earlier dependencies
// (:4598-4611 -> _transitions): the runnable new tasks recommended waiting in the dict's
// order (priority descending, popped LIFO), through the worker-loss recommendation machine
// (k_ev_lose_worker with no worker), every set order the cascade follows from the host
static int graph_stimulus_recompute(dgp_engine* e, int64_t n_order, const int32_t* order_task, const int8_t* order_kind,
                                    const int64_t* order_ptr, const int32_t* order_idx, int64_t* n_new_placements) {
  if (int rc = check_order_rows(e, n_order, order_task, order_kind, order_ptr, order_idx, "dgp_graph_stimulus_ordered"))
    return rc;
  dgp::Dev& D = e->D;
  const int64_t lo = e->pending_lo, N = D.N;
  std::vector<int32_t> recs;
  for (int64_t t = lo; t < N; t++) recs.push_back((int32_t)t);
  std::stable_sort(recs.begin(), recs.end(), [&](int32_t a, int32_t b) { return e->h_prio[a] > e->h_prio[b]; });
  int64_t pmax_old = -1;
  for (int64_t t = 0; t < lo; t++) pmax_old = std::max(pmax_old, e->h_prio[t]);
  bool follows = true;
  for (int64_t t = lo; t < N && follows; t++) follows = e->h_prio[t] > pmax_old;
  e->pending_resync = false;
  e->pending_lo = -1;
  e->mode = 2;
  HIPCHK(e, hipMemsetAsync(D.ready_key, 0xff, (size_t)D.N * 8, e->stream));  // the recommendation dict: empty
  std::vector<char*> a;
  const int64_t n_oidx = n_order ? order_ptr[n_order] : 0;
  if (int rc = stage_args(e, {{recs.data(), recs.size() * 4}, {order_task, (size_t)n_order * 4},
                              {order_kind, (size_t)n_order}, {order_ptr, n_order ? (size_t)(n_order + 1) * 8 : 0},
                              {order_idx, (size_t)n_oidx * 4}},
                          a))
    return rc;
  dgp::ev::LossOrder O{(const int32_t*)a[1], (const int8_t*)a[2], (const int64_t*)a[3], (const int32_t*)a[4],
                       (int)n_order};
  if (int rc = grow_logs(e, 0)) return rc;
  if (int rc = sync_dev(e)) return rc;
  dgp::Ctl c0;
  if (int rc = read_ctl(e, &c0)) return rc;
  hipLaunchKernelGGL(dgp::ev::k_ev_lose_worker, dim3(1), dim3(dgp::CTA), 0, e->stream, e->d_dev, (int)dgp::ev::LM_GRAPH,
                     -1, (const int32_t*)a[0], (int)recs.size(), (const int8_t*)nullptr, (const int32_t*)nullptr, 0, O,
                     e->d_aux + 3);
  HIPCHK(e, hipGetLastError());
  if (int rc = set_runids(e)) return rc;
  dgp::Ctl c;
  if (int rc = check_device_error(e, &c)) {
    e->pending_resync = true;  // the cascade stopped part-way: the scheduler's state is handed over
    return c.error == dgp::ERR_UNSUPPORTED ? fail(e, DGP_E_UNSUPPORTED, std::string(e->err)) : rc;
  }
  if (!follows && c.qlen > 1) {  // the queue (HeapSet by priority) with the new root-ish tasks in their place
    std::vector<int32_t> q((size_t)c.qlen);
    HIPCHK(e, hipMemcpy(q.data(), D.qarr + c.qhead, q.size() * 4, hipMemcpyDeviceToHost));
    std::stable_sort(q.begin(), q.end(), [&](int32_t x, int32_t y) { return e->h_prio[x] < e->h_prio[y]; });
    HIPCHK(e, hipMemcpy(D.qarr + c.qhead, q.data(), q.size() * 4, hipMemcpyHostToDevice));
  }
  if (n_new_placements) *n_new_placements = (int64_t)(c.n_placed - c0.n_placed);
  e->last_placed = c.n_placed;
  return 0;
}

int dgp_reschedule(dgp_engine* e, int32_t task, int64_t* n_new_placements) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (n_new_placements) *n_new_placements = 0;
  if (int rc = event_ready(e, "dgp_reschedule")) return rc;
  dgp::Dev& D = e->D;
  if (task < 0 || task >= D.N) return fail(e, DGP_E_ARG, "dgp_reschedule: task out of range");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, hipMemsetAsync(D.ready_key, 0xff, (size_t)D.N * 8, e->stream));  // the recommendation dict: empty
  std::vector<char*> a;
  if (int rc = stage_args(e, {{&task, 4}}, a)) return rc;
  if (int rc = grow_logs(e, 0)) return rc;
  if (int rc = sync_dev(e)) return rc;
  dgp::Ctl c0;
  if (int rc = read_ctl(e, &c0)) return rc;
  const dgp::ev::LossOrder O{nullptr, nullptr, nullptr, nullptr, 0};
  hipLaunchKernelGGL(dgp::ev::k_ev_lose_worker, dim3(1), dim3(dgp::CTA), 0, e->stream, e->d_dev,
                     (int)dgp::ev::LM_RELEASE, -1, (const int32_t*)a[0], 1, (const int8_t*)nullptr,
                     (const int32_t*)nullptr, 0, O, e->d_aux + 3);
  HIPCHK(e, hipGetLastError());
  if (int rc = set_runids(e)) return rc;
  dgp::Ctl c;
  if (int rc = check_device_error(e, &c)) {
    e->pending_resync = true;  // the cascade stopped part-way: the scheduler's state is handed over
    return c.error == dgp::ERR_UNSUPPORTED ? fail(e, DGP_E_UNSUPPORTED, std::string(e->err)) : rc;
  }
  if (n_new_placements) *n_new_placements = (int64_t)(c.n_placed - c0.n_placed);
  e->last_placed = c.n_placed;
  return 0;
}

int dgp_lose_worker(dgp_engine* e, int32_t worker, int64_t n_processing, const int32_t* processing, int64_t n_held,
                    const int32_t* held, int64_t* n_new_placements) {
  return dgp_lose_worker_ordered(e, worker, n_processing, processing, nullptr, n_held, held, 0, nullptr, nullptr,
                                 nullptr, nullptr, n_new_placements);
}

int dgp_lose_worker_ordered(dgp_engine* e, int32_t worker, int64_t n_processing, const int32_t* processing,
                            const int8_t* killed, int64_t n_held, const int32_t* held, int64_t n_order,
                            const int32_t* order_task, const int8_t* order_kind, const int64_t* order_ptr,
                            const int32_t* order_idx, int64_t* n_new_placements) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (n_new_placements) *n_new_placements = 0;
  if (int rc = event_ready(e, "dgp_lose_worker")) return rc;
  if (int rc = check_order_rows(e, n_order, order_task, order_kind, order_ptr, order_idx, "dgp_lose_worker_ordered"))
    return rc;
  dgp::Dev& D = e->D;
  if (worker < 0 || worker >= D.W) return fail(e, DGP_E_ARG, "dgp_lose_worker: worker out of range");
  if (e->paused_h[worker] == 2) return fail(e, DGP_E_ARG, "dgp_lose_worker: the worker was removed");
  if (n_processing < 0 || n_held < 0 || n_processing > D.N || n_held > D.N || (n_processing && !processing) ||
      (n_held && !held))
    return fail(e, DGP_E_ARG, "dgp_lose_worker: bad task lists");
  for (int64_t i = 0; i < n_processing; i++)
    if (processing[i] < 0 || processing[i] >= D.N) return fail(e, DGP_E_ARG, "dgp_lose_worker: task out of range");
  for (int64_t i = 0; i < n_held; i++)
    if (held[i] < 0 || held[i] >= D.N) return fail(e, DGP_E_ARG, "dgp_lose_worker: task out of range");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  // Scheduler.remove_worker's host part (:5217-5218): total_nthreads, which is_rootish reads
  e->paused_h[worker] = 2;
  D.total_nthreads -= e->nthreads[worker];
  D.evf |= dgp::EVF_PAUSED;
  if (int rc = refresh_rootish(e)) return rc;
  HIPCHK(e, hipMemsetAsync(D.ready_key, 0xff, (size_t)D.N * 8, e->stream));  // the recommendation dict: empty
  std::vector<char*> a;
  const int64_t n_oidx = n_order ? order_ptr[n_order] : 0;
  if (int rc = stage_args(e, {{processing, (size_t)n_processing * 4}, {held, (size_t)n_held * 4},
                              {order_task, (size_t)n_order * 4}, {order_kind, (size_t)n_order},
                              {order_ptr, n_order ? (size_t)(n_order + 1) * 8 : 0}, {order_idx, (size_t)n_oidx * 4},
                              {killed, killed ? (size_t)n_processing : 0}},
                          a))
    return rc;
  dgp::ev::LossOrder O{(const int32_t*)a[2], (const int8_t*)a[3], (const int64_t*)a[4], (const int32_t*)a[5],
                       (int)n_order};
  if (int rc = grow_logs(e, 0)) return rc;
  if (int rc = sync_dev(e)) return rc;
  hipLaunchKernelGGL(dgp::ev::k_ev_lose_worker, dim3(1), dim3(dgp::CTA), 0, e->stream, e->d_dev, (int)dgp::ev::LM_LOSS,
                     worker,
                     (const int32_t*)a[0], (int)n_processing, killed ? (const int8_t*)a[6] : nullptr,
                     (const int32_t*)a[1], (int)n_held, O, e->d_aux + 3);
  HIPCHK(e, hipGetLastError());
  if (int rc = set_runids(e)) return rc;
  long long placed = 0;
  HIPCHK(e, hipMemcpyAsync(&placed, e->d_aux + 3, sizeof placed, hipMemcpyDeviceToHost, e->stream));
  dgp::Ctl c;
  if (int rc = check_device_error(e, &c)) {
    // the cascade stopped part-way: the engine's state is the scheduler's to hand over
    e->pending_resync = true;
    return c.error == dgp::ERR_UNSUPPORTED ? fail(e, DGP_E_UNSUPPORTED, std::string(e->err)) : rc;
  }
  if (n_new_placements) *n_new_placements = placed;
  e->last_placed = c.n_placed;
  return 0;
}

int dgp_sync_placements(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker, const int64_t* comm_bytes,
                        const double* start_time, const int64_t* ws_nbytes, const int8_t* route) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (int rc = event_ready(e, "dgp_sync_placements")) return rc;
  if (n < 0 || (n > 0 && (!task || !worker || !comm_bytes || !start_time || !ws_nbytes || !route)))
    return fail(e, DGP_E_ARG, "dgp_sync_placements: bad batch");
  if (n == 0) return 0;
  dgp::Ctl c;
  if (int rc = read_ctl(e, &c)) return rc;
  e->last_placed = c.n_placed;
  if (int rc = grow_logs(e, 0)) return rc;
  if ((int64_t)c.n_placed + n > e->D.pl_cap) return fail(e, DGP_E_ARG, "dgp_sync_placements: more placements than tasks");
  for (int64_t i = 0; i < n; i++)
    if (task[i] < 0 || task[i] >= e->D.N || worker[i] < 0 || worker[i] >= e->D.W)
      return fail(e, DGP_E_ARG, "dgp_sync_placements: task or worker out of range");
  std::vector<char*> a;
  if (int rc = stage_args(e, {{task, n * 4}, {worker, n * 4}, {comm_bytes, n * 8}, {start_time, n * 8},
                              {ws_nbytes, n * 8}, {route, (size_t)n}}, a))
    return rc;
  if (int rc = sync_dev(e)) return rc;
  hipLaunchKernelGGL(dgp::ev::k_sync_placements, dim3(1), dim3(256), 0, e->stream, e->d_dev, (const int32_t*)a[0],
                     (const int32_t*)a[1], (const int64_t*)a[2], (const double*)a[3], (const int64_t*)a[4],
                     (const int8_t*)a[5], (int)n);
  HIPCHK(e, hipGetLastError());
  if (int rc = check_device_error(e, &c)) return rc;
  e->last_placed = c.n_placed;
  return 0;
}

int dgp_sync_tasks(dgp_engine* e, int64_t n, const int32_t* task, const uint8_t* state, const int32_t* remaining,
                   const int32_t* waiters, const int32_t* processing_on, const int64_t* nbytes,
                   const uint8_t* long_running, const uint8_t* wanted, const int64_t* holder_ptr,
                   const int32_t* holder_idx) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (int rc = event_ready(e, "dgp_sync_tasks")) return rc;
  if (n < 0 || (n > 0 && (!task || !state || !remaining || !waiters || !processing_on || !nbytes || !long_running ||
                          !wanted || !holder_ptr)))
    return fail(e, DGP_E_ARG, "dgp_sync_tasks: bad rows");
  if (n == 0) return 0;
  const dgp::Dev& D = e->D;
  const int64_t H = holder_ptr[n];
  if (holder_ptr[0] != 0 || H < 0 || (H > 0 && !holder_idx)) return fail(e, DGP_E_ARG, "dgp_sync_tasks: holder_ptr");
  std::vector<dgp::ev::SyncTask> rows(n);
  bool lr = false, multi = false;
  for (int64_t i = 0; i < n; i++) {
    const int32_t t = task[i];
    if (t < 0 || t >= D.N || state[i] > dgp::S_ERRED + 1 || holder_ptr[i + 1] < holder_ptr[i])
      return fail(e, DGP_E_ARG, "dgp_sync_tasks: task / state / holder_ptr");
    if (state[i] == dgp::S_PROCESSING && (processing_on[i] < 0 || processing_on[i] >= D.W))
      return fail(e, DGP_E_ARG, "dgp_sync_tasks: processing task without a worker");
    for (int64_t k = holder_ptr[i]; k < holder_ptr[i + 1]; k++)
      if (holder_idx[k] < 0 || holder_idx[k] >= D.W) return fail(e, DGP_E_ARG, "dgp_sync_tasks: holder out of range");
    auto& r = rows[i];
    r = dgp::ev::SyncTask{};
    r.t = t;
    r.proc_on = state[i] == dgp::S_PROCESSING ? processing_on[i] : -1;
    r.remaining = remaining[i];
    r.waiters = waiters[i];
    r.nbytes = nbytes[i];
    r.hp = (int32_t)holder_ptr[i];
    r.hn = (int32_t)(holder_ptr[i + 1] - holder_ptr[i]);
    // state 7 = forgotten (:2853): the row stays, released, flagged so that nothing walks it as
    // a dependent any more (_propagate_forgotten drops it from its dependencies' dependents)
    const bool forgotten = state[i] == dgp::S_ERRED + 1;
    r.state = forgotten ? (uint8_t)dgp::S_RELEASED : state[i];
    r.lr = long_running[i] ? 1 : 0;
    lr = lr || r.lr;
    multi = multi || r.hn > 1;
    // who_wants (TF_WANTED) rides on the host copy of the task flags
    e->tflags_h[t] = (uint8_t)((e->tflags_h[t] & ~(dgp::TF_WANTED | dgp::TF_FORGOTTEN)) |
                               (wanted[i] ? dgp::TF_WANTED : 0) | (forgotten ? dgp::TF_FORGOTTEN : 0));
    e->h_wanted[t] = wanted[i] ? 1 : 0;
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, hipMemcpy(const_cast<uint8_t*>(D.tflags), e->tflags_h.data(), D.N, hipMemcpyHostToDevice));
  std::vector<char*> a;
  if (int rc = stage_args(e, {{rows.data(), rows.size() * sizeof(dgp::ev::SyncTask)}, {holder_idx, (size_t)H * 4}}, a))
    return rc;
  // every resync may leave replica rows and long-running tasks: the paths that honour them stay on
  e->D.evf |= dgp::EVF_MULTI | (lr ? dgp::EVF_LR : 0);
  (void)multi;
  if (int rc = sync_dev(e)) return rc;
  hipLaunchKernelGGL(dgp::ev::k_sync_tasks, dim3(grid_for(n, 256, 1024)), dim3(256), 0, e->stream, e->d_dev,
                     (const dgp::ev::SyncTask*)a[0], (int)n, (const int32_t*)a[1]);
  HIPCHK(e, hipGetLastError());
  return check_device_error(e);
}

int dgp_sync_workers(dgp_engine* e, int32_t n_workers, const int8_t* status, const int32_t* nproc,
                     const int32_t* n_long_running, const int32_t* plen, const int32_t* prefix, const int32_t* count,
                     const int64_t* netocc, const int64_t* nbytes, const uint8_t* idle, const uint8_t* saturated,
                     const int64_t* needs_ptr, const int32_t* needs_task, const int32_t* needs_count) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (int rc = event_ready(e, "dgp_sync_workers")) return rc;
  dgp::Dev& D = e->D;
  namespace S = dgp::st;
  const int W = D.W;
  if (n_workers != W || !status || !nproc || !n_long_running || !plen || !prefix || !count || !netocc || !nbytes ||
      !idle || !saturated || !needs_ptr)
    return fail(e, DGP_E_ARG, "dgp_sync_workers: one row per engine worker");
  std::vector<int32_t> cap(W), pf((size_t)W * dgp::PMAX, 0), pc((size_t)W * dgp::PMAX, 0), pl(W);
  std::vector<uint8_t> fl(W);
  std::vector<int64_t> slots(W, 0);
  std::vector<uint32_t> lines((size_t)W * S::NLW, 0), ext((size_t)W * S::NXW, 0);
  int64_t n_idle = 0, n_sat = 0, n_itc = 0, itc_slots = 0;
  bool paused_any = false, lr_any = false;
  for (int w = 0; w < W; w++) {
    if (status[w] < 0 || status[w] > 2) return fail(e, DGP_E_ARG, "dgp_sync_workers: status");
    if (plen[w] < 0 || plen[w] > S::PD) return fail(e, DGP_E_ARG, "dgp_sync_workers: more than 8 prefixes on a worker");
    const bool running = status[w] == 0;
    if (!running && (idle[w] || saturated[w]))
      return fail(e, DGP_E_ARG, "dgp_sync_workers: a worker that is not running is neither idle nor saturated");
    if (status[w] == 2 && e->paused_h[w] != 2) D.total_nthreads -= e->nthreads[w];  // removed (:5217)
    if (status[w] != 2 && e->paused_h[w] == 2) return fail(e, DGP_E_ARG, "dgp_sync_workers: a removed worker returns");
    e->paused_h[w] = (uint8_t)status[w];
    paused_any = paused_any || !running;
    lr_any = lr_any || n_long_running[w] > 0;
    const int32_t nt = std::max<int32_t>(e->nthreads[w], 1);
    const int32_t base = D.sat_inf ? 0 : std::max((int32_t)std::ceil(D.saturation * nt), (int32_t)1);
    cap[w] = base + (D.sat_inf ? 0 : n_long_running[w]);
    pl[w] = plen[w];
    for (int i = 0; i < plen[w]; i++) {
      if (prefix[(size_t)w * S::PD + i] < 0 || prefix[(size_t)w * S::PD + i] >= D.P)
        return fail(e, DGP_E_ARG, "dgp_sync_workers: prefix id");
      pf[(size_t)w * dgp::PMAX + i] = prefix[(size_t)w * S::PD + i];
      pc[(size_t)w * dgp::PMAX + i] = count[(size_t)w * S::PD + i];
    }
    const bool itc = running && (D.sat_inf || cap[w] - nproc[w] > 0);
    fl[w] = (uint8_t)((idle[w] ? dgp::WF_IDLE : 0) | (saturated[w] ? dgp::WF_SAT : 0) | (itc ? dgp::WF_ITC : 0) |
                      (running ? 0 : dgp::WF_PAUSED));
    slots[w] = itc && !D.sat_inf ? cap[w] - nproc[w] : 0;
    n_idle += idle[w] ? 1 : 0;
    n_sat += saturated[w] ? 1 : 0;
    n_itc += itc ? 1 : 0;
    itc_slots += slots[w];
    // needs_what: up to NLW - 1 entries in the line, then NXW overflow entries, then scan mode
    const int64_t k0 = needs_ptr[w], k1 = needs_ptr[w + 1];
    const int64_t m = k1 - k0;
    if (k1 < k0 || (m > 0 && (!needs_task || !needs_count))) return fail(e, DGP_E_ARG, "dgp_sync_workers: needs_ptr");
    uint32_t* L = lines.data() + (size_t)w * S::NLW;
    if (m > (S::NLW - 1) + S::NXW) {
      L[S::NLW - 1] = S::NL_OVF;
    } else {
      for (int64_t k = 0; k < m; k++) {
        const int32_t d = needs_task[k0 + k], c = needs_count[k0 + k];
        if (d < 0 || d >= D.N || c <= 0 || c > 255) return fail(e, DGP_E_ARG, "dgp_sync_workers: needs_what entry");
        const uint32_t v = ((uint32_t)d << 8) | (uint32_t)c;
        if (k < S::NLW - 1) L[k] = v;
        else ext[(size_t)w * S::NXW + (k - (S::NLW - 1))] = v;
      }
      L[S::NLW - 1] = ((uint32_t)m << 8) | (m > S::NLW - 1 ? 1u : 0u);
    }
  }
  // is_rootish (:2929-2947) follows total_nthreads
  {
    std::vector<uint8_t>& tf = e->tflags_h;
    for (int64_t t = 0; t < D.N; t++) {
      const int g = e->group_h[t];
      const bool gr = e->group_sizes[g] > D.total_nthreads * 2 && e->gdep_n[g] < 5 && e->gdep_len[g] < 5;
      const bool rs = !e->restr_h.empty() && (e->restr_h[t] & dgp::RF_RESTRICTED);
      const bool r = e->rootish_override_h[t] >= 0 ? e->rootish_override_h[t] != 0 : (gr && !rs);
      tf[t] = (uint8_t)((tf[t] & ~dgp::TF_ROOTISH) | (r ? dgp::TF_ROOTISH : 0));
    }
  }
  HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, hipMemcpy(const_cast<uint8_t*>(D.tflags), e->tflags_h.data(), D.N, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_cap, cap.data(), (size_t)W * 4, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_nproc, nproc, (size_t)W * 4, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_plen, pl.data(), (size_t)W * 4, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_pfx, pf.data(), pf.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_pcnt, pc.data(), pc.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_netocc, netocc, (size_t)W * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_nbytes, nbytes, (size_t)W * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_flags, fl.data(), (size_t)W, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_itcslots, slots.data(), (size_t)W * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.gw_needs_saved, lines.data(), lines.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.gw_needs_ext, ext.data(), ext.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.w_nthreads, e->nthreads.data(), (size_t)W * 4, hipMemcpyHostToDevice));
  dgp::Ctl c;
  if (int rc = read_ctl(e, &c)) return rc;
  c.n_idle = n_idle;
  c.n_sat = n_sat;
  c.n_itc = n_itc;
  c.itc_slots = itc_slots;
  HIPCHK(e, hipMemcpy(e->ctl, &c, sizeof c, hipMemcpyHostToDevice));
  if (paused_any) D.evf |= dgp::EVF_PAUSED;
  if (lr_any) D.evf |= dgp::EVF_LR;
  return sync_dev(e);
}

int dgp_sync_globals(dgp_engine* e, int64_t n_tasks_counter, double network_occ_global, int32_t g_plen,
                     const int32_t* g_prefix, const int64_t* g_count, int64_t n_queued, const int32_t* queued,
                     const double* duration_average, const double* max_exec_time, double bandwidth,
                     const int64_t* group_released_waiting, const int64_t* group_left, const int32_t* group_last_worker) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (int rc = event_ready(e, "dgp_sync_globals")) return rc;
  dgp::Dev& D = e->D;
  if (g_plen < 0 || g_plen > dgp::PMAX_G || (g_plen > 0 && (!g_prefix || !g_count)) || n_queued < 0 ||
      n_queued > D.N || (n_queued > 0 && !queued) || !duration_average || !max_exec_time || !(bandwidth > 0) ||
      !group_released_waiting || !group_left || !group_last_worker)
    return fail(e, DGP_E_ARG, "dgp_sync_globals: bad arguments");
  for (int i = 0; i < g_plen; i++)
    if (g_prefix[i] < 0 || g_prefix[i] >= D.P) return fail(e, DGP_E_ARG, "dgp_sync_globals: prefix id");
  for (int64_t i = 0; i < n_queued; i++)
    if (queued[i] < 0 || queued[i] >= D.N) return fail(e, DGP_E_ARG, "dgp_sync_globals: queued task");
  for (int g = 0; g < D.G; g++)
    if (group_last_worker[g] < -1 || group_last_worker[g] >= D.W) return fail(e, DGP_E_ARG, "dgp_sync_globals: last worker");
  HIPCHK(e, hipStreamSynchronize(e->stream));
  dgp::Ctl c;
  if (int rc = read_ctl(e, &c)) return rc;
  c.n_tasks = n_tasks_counter;
  c.g_netocc = network_occ_global;
  c.g_plen = g_plen;
  for (int i = 0; i < dgp::PMAX_G; i++) {
    c.g_pfx[i] = i < g_plen ? g_prefix[i] : 0;
    c.g_pcnt[i] = i < g_plen ? g_count[i] : 0;
  }
  c.qhead = 0;
  c.qlen = n_queued;
  HIPCHK(e, hipMemcpy(e->ctl, &c, sizeof c, hipMemcpyHostToDevice));
  if (n_queued) HIPCHK(e, hipMemcpy(D.qarr, queued, n_queued * 4, hipMemcpyHostToDevice));
  for (double* p : {D.pdur_cur, D.pdur_walk, D.pdur_pre})
    HIPCHK(e, hipMemcpy(p, duration_average, (size_t)D.P * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.pmaxexec, max_exec_time, (size_t)D.P * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.g_relwait, group_released_waiting, (size_t)D.G * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.g_left, group_left, (size_t)D.G * 8, hipMemcpyHostToDevice));
  HIPCHK(e, hipMemcpy(D.g_lastw, group_last_worker, (size_t)D.G * 4, hipMemcpyHostToDevice));
  D.bandwidth = bandwidth;
  if (int rc = sync_dev(e)) return rc;
  e->pending_resync = false;  // the resync is complete (dgp_sync_globals comes last)
  e->pending_lo = -1;
  return 0;
}

int dgp_snapshot(dgp_engine* e) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (e->snap_rounds <= 0) return fail(e, DGP_E_STATE, "snapshots not enabled");
  HIPCHK(e, hipSetDevice(e->device));
  hipLaunchKernelGGL(dgp::svc::k_svc_snapshot_begin, dim3(1), dim3(64), 0, e->stream, e->d_dev);
  hipLaunchKernelGGL(dgp::k_snapshot, dim3(8), dim3(256), 0, e->stream, e->d_dev, e->d_aux + 1, 0);
  HIPCHK(e, hipGetLastError());
  return check_device_error(e);
}

int64_t dgp_num_placements(dgp_engine* e) {
  if (!e) return -1;
  if (e->posted) {
    fail(e, DGP_E_STATE, "a posted task-finished batch: dgp_tasks_finished_wait first");
    return -1;
  }
  // the resident kernel publishes the log length with every answer
  if (e->res_running) return __atomic_load_n(&e->mb->n_placed, __ATOMIC_ACQUIRE);
  dgp::Ctl c;
  if (read_ctl(e, &c)) return -1;
  return (int64_t)c.n_placed;
}

int dgp_get_placements(dgp_engine* e, int64_t offset, int64_t count, int32_t* task, int32_t* worker,
                       int64_t* comm_bytes, double* start_time, int64_t* ws_nbytes, int8_t* route) {
  if (!e || offset < 0 || count < 0) return fail(e, DGP_E_ARG, "bad range");
  if (e->posted) return fail(e, DGP_E_STATE, "a posted task-finished batch: dgp_tasks_finished_wait first");
  if (e->res_running) {  // the last answer's new placements are in the mailbox (task / worker)
    const int64_t a = e->mb->pl_from, b = e->mb->n_placed;
    if (a >= 0 && offset >= a && offset + count <= b && !comm_bytes && !start_time && !ws_nbytes && !route) {
      if (task) memcpy(task, dgp::svc::mbox_pl_task(e->mb) + (offset - a), (size_t)count * 4);
      if (worker) memcpy(worker, dgp::svc::mbox_pl_worker(e->mb) + (offset - a), (size_t)count * 4);
      return 0;
    }
    if (int rc = resident_stop(e)) return rc;
  }
  int64_t n = dgp_num_placements(e);
  if (n < 0) return DGP_E_HIP;
  if (offset + count > n) return fail(e, DGP_E_ARG, "range beyond the placement log");
  if (count == 0) return 0;
  const dgp::Dev& D = e->D;
  auto cp = [&](void* dst, const void* src, size_t sz) {  // queued on the engine's stream, one sync below
    return dst ? hipMemcpyAsync(dst, (const char*)src + offset * sz, count * sz, hipMemcpyDeviceToHost, e->stream)
               : hipSuccess;
  };
  HIPCHK(e, cp(task, D.pl_task, 4));
  HIPCHK(e, cp(worker, D.pl_worker, 4));
  HIPCHK(e, cp(comm_bytes, D.pl_comm, 8));
  HIPCHK(e, cp(start_time, D.pl_start, 8));
  HIPCHK(e, cp(ws_nbytes, D.pl_wsnbytes, 8));
  HIPCHK(e, cp(route, D.pl_route, 1));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return 0;
}

int dgp_task_messages(dgp_engine* e, int64_t offset, int64_t count, int64_t* n_deps, int64_t* n_holders,
                      int64_t* dep_ptr, int32_t* dep_task, int64_t* dep_nbytes, int64_t* holder_ptr,
                      int32_t* holder_idx) {
  if (e && e->posted) return fail(e, DGP_E_STATE, "a posted task-finished batch: dgp_tasks_finished_wait first");
  if (e && e->res_running && n_deps && n_holders && offset >= 0 && count >= 0) {
    // the last resident answer's placements: their fields are in the mailbox (dgp_set_task_messages)
    namespace V = dgp::svc;
    V::Mbox* m = e->mb;
    const int64_t a = m->msg_from, b = m->n_placed;
    if (a >= 0 && offset >= a && offset + count <= b) {
      const int32_t* dp = V::mbox_m_dptr(m) + (offset - a);
      const int32_t* hp = V::mbox_m_hptr(m);
      const int64_t d0 = dp[0], d1 = dp[count], h0 = hp[d0], h1 = hp[d1];
      *n_deps = d1 - d0;
      *n_holders = h1 - h0;
      if (!dep_ptr) return 0;  // size query
      if (!dep_task || !dep_nbytes || !holder_ptr || (h1 > h0 && !holder_idx))
        return fail(e, DGP_E_ARG, "dgp_task_messages: output arrays missing");
      for (int64_t j = 0; j <= count; j++) dep_ptr[j] = dp[j] - d0;
      for (int64_t k = d0; k <= d1; k++) holder_ptr[k - d0] = hp[k] - h0;
      if (d1 > d0) {
        memcpy(dep_task, V::mbox_m_dtask(m) + d0, (size_t)(d1 - d0) * 4);
        memcpy(dep_nbytes, V::mbox_m_dnb(m) + d0, (size_t)(d1 - d0) * 8);
      }
      if (h1 > h0) memcpy(holder_idx, V::mbox_m_hidx(m) + h0, (size_t)(h1 - h0) * 4);
      return 0;
    }
  }
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->graph_done) return fail(e, DGP_E_STATE, "dgp_update_graph first");
  if (offset < 0 || count < 0 || !n_deps || !n_holders) return fail(e, DGP_E_ARG, "dgp_task_messages: bad arguments");
  const int64_t n = dgp_num_placements(e);
  if (n < 0) return DGP_E_HIP;
  if (offset + count > n) return fail(e, DGP_E_ARG, "dgp_task_messages: range beyond the placement log");
  if (count > INT32_MAX / 2) return fail(e, DGP_E_ARG, "dgp_task_messages: batch too large");
  HIPCHK(e, hipSetDevice(e->device));
  *n_deps = *n_holders = 0;
  if (count == 0) {
    if (dep_ptr) dep_ptr[0] = 0;
    if (holder_ptr) holder_ptr[0] = 0;
    return 0;
  }
  auto grow = [&](size_t need) -> int {
    if (need <= e->d_msgbuf_cap) return 0;
    if (e->d_msgbuf) (void)hipFree(e->d_msgbuf);
    e->d_msgbuf = nullptr;
    e->d_msgbuf_cap = 0;
    const size_t cap = std::max(need, (size_t)1 << 20);
    HIPCHK(e, hipMalloc((void**)&e->d_msgbuf, cap));
    e->d_msgbuf_cap = cap;
    return 0;
  };
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  // pass 1: per placement, its dependencies and their holders
  const size_t c = (size_t)count;
  if (int rc = grow(2 * al(c * 4))) return rc;
  int32_t* d_nd = (int32_t*)e->d_msgbuf;
  int32_t* d_nh = (int32_t*)(e->d_msgbuf + al(c * 4));
  hipStream_t s = e->stream;
  if (int rc = sync_dev(e)) return rc;
  hipLaunchKernelGGL(dgp::msg::k_msg_count, dim3((unsigned)((c + 255) / 256)), dim3(256), 0, s, e->d_dev,
                     (long long)offset, (int)count, d_nd, d_nh);
  HIPCHK(e, hipGetLastError());
  std::vector<int32_t> nd(c), nh(c);
  HIPCHK(e, hipMemcpyAsync(nd.data(), d_nd, c * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(e, hipMemcpyAsync(nh.data(), d_nh, c * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(e, hipStreamSynchronize(s));
  std::vector<int64_t> dp(c + 1, 0), hb(c + 1, 0);
  for (size_t j = 0; j < c; j++) {
    dp[j + 1] = dp[j] + nd[j];
    hb[j + 1] = hb[j] + nh[j];
  }
  *n_deps = dp[c];
  *n_holders = hb[c];
  if (!dep_ptr) return 0;  // size query
  if (!dep_task || !dep_nbytes || !holder_ptr || (hb[c] > 0 && !holder_idx))
    return fail(e, DGP_E_ARG, "dgp_task_messages: output arrays missing");
  memcpy(dep_ptr, dp.data(), (c + 1) * 8);
  const size_t E = (size_t)dp[c], H = (size_t)hb[c];
  // pass 2: the rows, at the scanned offsets
  const size_t o_dp = 0, o_hb = o_dp + al((c + 1) * 8), o_task = o_hb + al((c + 1) * 8), o_nb = o_task + al(E * 4),
               o_hc = o_nb + al(E * 8), o_hi = o_hc + al(E * 4), total = o_hi + al(H * 4);
  if (int rc = grow(total)) return rc;
  char* B = e->d_msgbuf;
  HIPCHK(e, hipMemcpyAsync(B + o_dp, dp.data(), (c + 1) * 8, hipMemcpyHostToDevice, s));
  HIPCHK(e, hipMemcpyAsync(B + o_hb, hb.data(), (c + 1) * 8, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(dgp::msg::k_msg_fill, dim3((unsigned)((c + 255) / 256)), dim3(256), 0, s, e->d_dev,
                     (long long)offset, (int)count, (const int64_t*)(B + o_dp), (const int64_t*)(B + o_hb),
                     (int32_t*)(B + o_task), (int64_t*)(B + o_nb), (int32_t*)(B + o_hc), (int32_t*)(B + o_hi));
  HIPCHK(e, hipGetLastError());
  std::vector<int32_t> hc(E);
  if (E) {
    HIPCHK(e, hipMemcpyAsync(dep_task, B + o_task, E * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(e, hipMemcpyAsync(dep_nbytes, B + o_nb, E * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(e, hipMemcpyAsync(hc.data(), B + o_hc, E * 4, hipMemcpyDeviceToHost, s));
  }
  if (H) HIPCHK(e, hipMemcpyAsync(holder_idx, B + o_hi, H * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(e, hipStreamSynchronize(s));
  holder_ptr[0] = 0;
  for (size_t k = 0; k < E; k++) holder_ptr[k + 1] = holder_ptr[k] + hc[k];
  return check_device_error(e);
}

int dgp_enable_snapshots(dgp_engine* e, int64_t max_rounds) {
  if (int rc_ = resident_stop(e)) return rc_;
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
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || e->snap_rounds <= 0) return fail(e, DGP_E_STATE, "snapshots not enabled");
  const dgp::Dev& D = e->D;
  dgp::Ctl c;
  if (int rc = read_ctl(e, &c)) return rc;
  int64_t R = std::min<int64_t>(e->graph_done ? c.rounds_nonempty + 1 : 0, e->snap_rounds);
  if (n_rounds) *n_rounds = R;
  if (R == 0) return 0;
  size_t RW = (size_t)R * D.W;
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
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->have_graph || !state) return fail(e, DGP_E_ARG, "graph first");
  HIPCHK(e, hipStreamSynchronize(e->stream));
  HIPCHK(e, hipMemcpy(state, e->D.state, e->D.N, hipMemcpyDeviceToHost));
  return 0;
}

int dgp_kernel_times(dgp_engine* e, double* ms, int64_t* launches, int32_t n) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e) return DGP_E_ARG;
  if (int rc = resolve_timing(e)) return rc;
  for (int k = 0; k < n && k < 8; k++) {
    if (ms) ms[k] = e->kms[k];
    if (launches) launches[k] = e->klaunch[k];
  }
  return 0;
}

int dgp_set_timing(dgp_engine* e, int enabled) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e) return DGP_E_ARG;
  e->timing = enabled != 0;
  return 0;
}

extern "C" int dgp_debug_trace(dgp_engine* e, unsigned long long* out) {  // DGP_TRACE builds
  if (!e || !e->D.trace) return DGP_E_ARG;
  HIPCHK(e, hipMemcpy(out, e->D.trace, e->D.trace_n * 32 * 8, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int dgp_debug_buf(dgp_engine* e, double* out) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !e->D.dbgbuf) return DGP_E_ARG;
  HIPCHK(e, hipMemcpy(out, e->D.dbgbuf, 64 * 8 * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

// Longest chain of the replay's conflict DAG (measurement; host code, no engine): stimulus r
// completes pl_task[r] (the replay completes tasks in run_id order, SURVEY.md §8 replay
// definition) and touches the completing worker, the holder of every dependency it
// releases (its last dependent completed, not wanted: scheduler.py:3309-3314) and the
// holder of every dependency of each task it makes ready (decide_worker's candidates,
// :8550-8593). Two stimuli that touch one worker are ordered; depth = 1 + the deepest
// earlier stimulus sharing a worker. Queue refills (rootish placements popped by a
// completion, :4983-5023) are not modelled, so depth is a lower bound on the ordered links.
int dgp_conflict_depth(int64_t n_tasks, const int64_t* dep_ptr, const int32_t* dep_idx, const uint8_t* wanted,
                       int64_t n_pl, const int32_t* pl_task, const int32_t* pl_worker, int64_t first,
                       int64_t* depth, int64_t* n_touch) {
  if (n_tasks < 0 || n_pl < 0 || n_pl > n_tasks || first < 0 || !depth || (n_tasks && (!dep_ptr || !wanted)) ||
      (n_pl && (!pl_task || !pl_worker)))
    return DGP_E_ARG;
  std::vector<int64_t> run(n_tasks, -1);
  std::vector<int32_t> holder(n_tasks, -1);
  int32_t wmax = 0;
  for (int64_t r = 0; r < n_pl; r++) {
    if (pl_task[r] < 0 || pl_task[r] >= n_tasks || pl_worker[r] < 0) return DGP_E_ARG;
    run[pl_task[r]] = r;
    holder[pl_task[r]] = pl_worker[r];
    wmax = std::max(wmax, pl_worker[r]);
  }
  std::vector<int64_t> fr(n_tasks, -1), rel(n_tasks, -1);  // frontier / release stimulus
  std::vector<uint8_t> has_dep(n_tasks, 0);
  for (int64_t x = 0; x < n_tasks; x++)
    for (int64_t j = dep_ptr[x]; j < dep_ptr[x + 1]; j++) {
      const int32_t d = dep_idx[j];
      fr[x] = std::max(fr[x], run[d]);
      rel[d] = std::max(rel[d], run[x]);
      has_dep[d] = 1;
    }
  std::vector<int64_t> cnt(n_pl + 1, 0);
  for (int64_t r = 0; r < n_pl; r++) cnt[r + 1]++;
  for (int64_t x = 0; x < n_tasks; x++) {
    if (fr[x] >= 0) cnt[fr[x] + 1] += dep_ptr[x + 1] - dep_ptr[x];
    if (has_dep[x] && !wanted[x] && rel[x] >= 0) cnt[rel[x] + 1]++;
  }
  for (int64_t r = 0; r < n_pl; r++) cnt[r + 1] += cnt[r];
  std::vector<int32_t> tw(cnt[n_pl]);
  std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
  for (int64_t r = 0; r < n_pl; r++) tw[pos[r]++] = pl_worker[r];
  for (int64_t x = 0; x < n_tasks; x++) {
    if (fr[x] >= 0)
      for (int64_t j = dep_ptr[x]; j < dep_ptr[x + 1]; j++) tw[pos[fr[x]]++] = holder[dep_idx[j]];
    if (has_dep[x] && !wanted[x] && rel[x] >= 0) tw[pos[rel[x]]++] = holder[x];
  }
  std::vector<int64_t> last(wmax + 1, 0);
  int64_t best = 0;
  for (int64_t r = first; r < n_pl; r++) {
    int64_t dp = 0;
    for (int64_t i = cnt[r]; i < cnt[r + 1]; i++)
      if (tw[i] >= 0) dp = std::max(dp, last[tw[i]]);
    dp += 1;
    for (int64_t i = cnt[r]; i < cnt[r + 1]; i++)
      if (tw[i] >= 0) last[tw[i]] = dp;
    best = std::max(best, dp);
  }
  *depth = best;
  if (n_touch) *n_touch = cnt[n_pl] - cnt[std::min(first, n_pl)];
  return 0;
}

int dgp_stats(dgp_engine* e, int64_t* out, int32_t n) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e || !out) return DGP_E_ARG;
  dgp::Ctl c;
  if (int rc = read_ctl(e, &c)) return rc;
  int64_t v[49] = {(int64_t)c.n_placed, c.rounds_nonempty, c.dr_steps, c.n_global_events, (int64_t)c.rec_used,
                   (int64_t)c.walk_pos};
  for (int i = 0; i < 8; i++) v[6 + i] = (int64_t)c.prof[i];
  for (int i = 0; i < 16; i++) v[14 + i] = (int64_t)c.prof2[i];
  for (int i = 0; i < 8; i++) v[30 + i] = (int64_t)c.prof3[i];
  for (int i = 0; i < 4; i++) v[38 + i] = e->res_prof[i];
  for (int i = 0; i < 7; i++) v[42 + i] = e->res_role[i];
  for (int i = 0; i < n && i < 49; i++) out[i] = v[i];
  return 0;
}


// ------------------------------------------------------------------ WorkStealing
// WorkStealing.balance (stealing.py:401-503) over host arrays (see include/dgplace.h).
// WorkStealing state resident in the engine between the phases of one balance():
// dgp_steal_load (upload, levels, bins, thief order) -> dgp_steal_thief_rows (any
// slice of the stealable positions; ranks of a sharded call each take one) ->
// [dgp_steal_pack_rows / dgp_steal_unpack_rows around an all-gather] -> dgp_steal_run.
int dgp_steal_load(dgp_engine* e, int32_t W, const int32_t* nthreads, const double* occ, const int32_t* nproc,
                   const int64_t* wnbytes, const uint8_t* idle, const uint8_t* sat, double total_occ,
                   int64_t total_nthreads, int64_t bandwidth, int64_t T, const int32_t* victim, const double* duration,
                   const uint8_t* fast, const int64_t* dep_ptr, const int32_t* dep_idx, int64_t n_data,
                   const int64_t* d_nbytes, const int64_t* d_get_nbytes, const int64_t* h_ptr, const int32_t* h_idx,
                   const int64_t* r_ptr, const int32_t* r_idx, const uint8_t* r_flags, const int8_t* level_in,
                   const double* ifo_in, const int32_t* ift_in, int64_t* n_stealable) {
  if (int rc_ = resident_stop(e)) return rc_;
  namespace S = dgp::steal;
  if (!e) return DGP_E_ARG;
  e->steal.loaded = false;
  if (W <= 0 || T < 0 || n_data < 0 || bandwidth <= 0 || total_nthreads <= 0 || !nthreads || !occ || !nproc ||
      !wnbytes || !idle || !sat || !n_stealable || (T && (!victim || !duration || !fast || !dep_ptr)) ||
      (n_data && (!d_nbytes || !d_get_nbytes || !h_ptr)))
    return fail(e, DGP_E_ARG, "dgp_steal_load: bad sizes or null pointers");
  if (S::balance_lds_bytes(W) > 160 * 1024) return fail(e, DGP_E_ARG, "dgp_steal_load: too many workers");
  for (int32_t w = 0; w < W; w++)  // k_balance keeps nthreads as uint16 in LDS
    if (nthreads[w] <= 0 || nthreads[w] > 65535) return fail(e, DGP_E_ARG, "dgp_steal_load: nthreads out of range");
  if ((size_t)W * S::N_LEVELS >= (1u << 30)) return fail(e, DGP_E_ARG, "dgp_steal_load: W too large");
  if (T >= (1ll << 31)) return fail(e, DGP_E_ARG, "dgp_steal_load: too many tasks");
  // the shapes the kernels assume, checked on the host
  for (int32_t w = 0; w < W; w++)
    if (nthreads[w] <= 0) return fail(e, DGP_E_ARG, "dgp_steal_load: nthreads must be positive");
  const int64_t E = T ? dep_ptr[T] : 0;
  if (T && (dep_ptr[0] != 0 || E < 0)) return fail(e, DGP_E_ARG, "dgp_steal_load: dep_ptr");
  if (E && !dep_idx) return fail(e, DGP_E_ARG, "dgp_steal_load: dep_idx");
  for (int64_t t = 0; t < T; t++) {
    if (victim[t] < 0 || victim[t] >= W) return fail(e, DGP_E_ARG, "dgp_steal_load: victim out of range");
    if (dep_ptr[t + 1] < dep_ptr[t]) return fail(e, DGP_E_ARG, "dgp_steal_load: dep_ptr not monotone");
  }
  for (int64_t k = 0; k < E; k++)
    if (dep_idx[k] < 0 || dep_idx[k] >= n_data) return fail(e, DGP_E_ARG, "dgp_steal_load: dep_idx out of range");
  const int64_t H = n_data ? h_ptr[n_data] : 0;
  if (n_data && h_ptr[0] != 0) return fail(e, DGP_E_ARG, "dgp_steal_load: h_ptr");
  for (int64_t d = 0; d < n_data; d++)
    if (h_ptr[d + 1] < h_ptr[d]) return fail(e, DGP_E_ARG, "dgp_steal_load: h_ptr not monotone");
  if (H && !h_idx) return fail(e, DGP_E_ARG, "dgp_steal_load: h_idx");
  const int64_t RK = r_flags ? (r_ptr ? r_ptr[T] : -1) : 0;
  if (level_in)
    for (int64_t t = 0; t < T; t++)
      if (level_in[t] < -1 || level_in[t] >= S::N_LEVELS) return fail(e, DGP_E_ARG, "dgp_steal_load: level_in");
  if (r_flags) {
    if (!r_ptr || r_ptr[0] != 0 || RK < 0 || (RK && !r_idx)) return fail(e, DGP_E_ARG, "dgp_steal_load: restrictions");
    for (int64_t t = 0; t < T; t++)
      if (r_ptr[t + 1] < r_ptr[t] || (r_flags[t] & ~3)) return fail(e, DGP_E_ARG, "dgp_steal_load: restrictions");
    for (int64_t k = 0; k < RK; k++)
      if (r_idx[k] < 0 || r_idx[k] >= W) return fail(e, DGP_E_ARG, "dgp_steal_load: restricted worker out of range");
  }
  for (int64_t k = 0; k < H; k++)
    if (h_idx[k] < 0 || h_idx[k] >= W) return fail(e, DGP_E_ARG, "dgp_steal_load: holder out of range");
  HIPCHK(e, hipSetDevice(e->device));
  hipStream_t s = e->stream;
  StealCtx& C = e->steal;
  const int NK = S::N_LEVELS * W + 1;
  std::vector<std::pair<void**, size_t>> parts;
  S::Prob P{};
  int32_t *d_nthreads, *d_nproc, *d_victim, *d_dep_idx, *d_h_idx;
  double *d_occ, *d_dur;
  int64_t *d_wnb, *d_dep_ptr, *d_dnb, *d_dgnb, *d_h_ptr;
  uint8_t *d_idle, *d_sat, *d_fast;
  const int Tn = (int)T;
  size_t tmp_sort = 0, tmp_scan = 0, tmp_nb = 0, tmp_a = 0;
  hipError_t st = hipSuccess;
  auto chk = [&](hipError_t x) {
    if (x != hipSuccess && st == hipSuccess) st = x;
  };
  chk(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_sort, (int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr,
                                         (int32_t*)nullptr, std::max(Tn, 1), 0, 32, s));
  chk(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_scan, (int32_t*)nullptr, (int32_t*)nullptr, NK, s));
  // the two stable sorts that order the initial thieves
  chk(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_nb, (int64_t*)nullptr, (int64_t*)nullptr, (int32_t*)nullptr,
                                         (int32_t*)nullptr, W, 0, 64, s));
  chk(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_a, (uint64_t*)nullptr, (uint64_t*)nullptr, (int32_t*)nullptr,
                                         (int32_t*)nullptr, W, 0, 64, s));
  // dgp_steal_order: the tasks' (priority, arrival) order, two stable 64-bit sorts
  const bool ordered = (int64_t)e->steal.order_prio.size() == T && T > 0;
  size_t tmp_ord = 0;
  if (ordered)
    chk(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_ord, (uint64_t*)nullptr, (uint64_t*)nullptr, (int32_t*)nullptr,
                                           (int32_t*)nullptr, Tn, 0, 64, s));
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("dgp_steal_load: sizing: ") + hipGetErrorString(st));
  const size_t tmp_bytes = std::max(std::max(std::max(tmp_sort, tmp_scan), std::max(tmp_nb, tmp_a)), tmp_ord);
  auto add = [&](auto** p, size_t n) { parts.push_back({(void**)p, (n ? n : 1) * sizeof(**p)}); };
  add(&d_nthreads, W); add(&d_occ, W); add(&d_nproc, W); add(&d_wnb, W); add(&d_idle, W); add(&d_sat, W);
  add(&d_victim, T); add(&d_dur, T); add(&d_fast, T); add(&d_dep_ptr, T + 1); add(&d_dep_idx, E);
  add(&d_dnb, n_data); add(&d_dgnb, n_data); add(&d_h_ptr, n_data + 1); add(&d_h_idx, H);
  int64_t* d_r_ptr = nullptr;
  int32_t* d_r_idx = nullptr;
  uint8_t* d_r_flags = nullptr;
  if (r_flags) {
    add(&d_r_ptr, T + 1); add(&d_r_idx, RK); add(&d_r_flags, T);
  }
  int8_t* d_lv_in = nullptr;
  double* d_ifo_in = nullptr;
  int32_t* d_ift_in = nullptr;
  if (level_in) add(&d_lv_in, T);
  if (ifo_in) add(&d_ifo_in, W);
  if (ift_in) add(&d_ift_in, W);
  add(&P.checked, W);
  uint64_t *d_ok1 = nullptr, *d_ok2 = nullptr, *d_ok3 = nullptr;
  int32_t *d_perm1 = nullptr, *d_perm2 = nullptr;
  if (ordered) {
    add(&d_ok1, T); add(&d_ok2, T); add(&d_ok3, T); add(&d_perm1, T); add(&d_perm2, T);
  }
  add(&P.key, T); add(&P.order, T); add(&C.keys_sorted, T); add(&C.d_vals, T); add(&P.bin_cnt, NK); add(&P.bin_ptr, NK);
  add(&P.s_best, T); add(&P.s_cct, T); add(&P.s_ccv, T); add(&P.s_dur, T);
  add(&P.s_cget, T); add(&P.s_craw, T); add(&P.s_nh, T); add(&P.s_hw, T * S::MAXH); add(&P.s_hg, T * S::MAXH);
  add(&P.s_hr, T * S::MAXH);
  add(&P.tk_a, W); add(&P.tk_nb, W); add(&P.tk_w, W); add(&P.tk_a2, W); add(&P.tk_nb2, W); add(&P.tk_w2, W);
  add(&P.th_order, W); add(&P.run_start, W + 1); add(&P.run_a, W); add(&P.run_of_w, W); add(&P.n_runs, 1);
  add(&P.vs_g, W);
  add(&P.level, T); add(&P.st_task, T); add(&P.st_victim, T); add(&P.st_thief, T); add(&P.st_level, T);
  add(&P.st_cost, T); add(&P.st_occ_victim, T); add(&P.st_occ_thief, T); add(&P.n_steals, 1);
  add(&P.inflight_occ, W); add(&P.inflight_tasks, W); add(&P.idle_out, W); add(&P.sat_out, W);
  size_t total = (tmp_bytes + 255) / 256 * 256;
  for (auto& pr : parts) total += (pr.second + 255) / 256 * 256;
  if (total > C.cap) {  // the arena grows, never shrinks, while the engine lives
    if (C.arena) HIPCHK(e, hipFree(C.arena));
    C.arena = nullptr;
    C.cap = 0;
    HIPCHK(e, hipMalloc(&C.arena, total));
    C.cap = total;
  }
  size_t off = 0;
  C.d_tmp = C.arena;
  C.tmp_bytes = tmp_bytes;
  off += (tmp_bytes + 255) / 256 * 256;
  for (auto& pr : parts) {
    *pr.first = C.arena + off;
    off += (pr.second + 255) / 256 * 256;
  }
  auto h2d = [&](void* dst, const void* src, size_t bytes) {
    return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s) : hipSuccess;
  };
  chk(h2d(d_nthreads, nthreads, W * 4)); chk(h2d(d_occ, occ, W * 8)); chk(h2d(d_nproc, nproc, W * 4));
  chk(h2d(d_wnb, wnbytes, W * 8)); chk(h2d(d_idle, idle, W)); chk(h2d(d_sat, sat, W));
  chk(h2d(d_victim, victim, T * 4)); chk(h2d(d_dur, duration, T * 8)); chk(h2d(d_fast, fast, T));
  chk(h2d(d_dep_ptr, dep_ptr, (T + 1) * 8)); chk(h2d(d_dep_idx, dep_idx, E * 4));
  chk(h2d(d_dnb, d_nbytes, n_data * 8)); chk(h2d(d_dgnb, d_get_nbytes, n_data * 8));
  chk(h2d(d_h_ptr, h_ptr, (n_data + 1) * 8)); chk(h2d(d_h_idx, h_idx, H * 4));
  if (r_flags) {
    chk(h2d(d_r_ptr, r_ptr, (T + 1) * 8)); chk(h2d(d_r_idx, r_idx, RK * 4)); chk(h2d(d_r_flags, r_flags, T));
  }
  chk(hipMemsetAsync(P.bin_cnt, 0, NK * 4, s));
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("dgp_steal_load: upload: ") + hipGetErrorString(st));
  if (level_in) chk(h2d(d_lv_in, level_in, T));
  if (ifo_in) chk(h2d(d_ifo_in, ifo_in, W * 8));
  if (ift_in) chk(h2d(d_ift_in, ift_in, W * 4));
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("dgp_steal_load: upload: ") + hipGetErrorString(st));
  P.r_ptr = d_r_ptr;
  P.r_idx = d_r_idx;
  P.r_flags = d_r_flags;
  P.level_in = d_lv_in;
  P.ifo_in = d_ifo_in;
  P.ift_in = d_ift_in;
  P.W = W; P.nthreads = d_nthreads; P.occ = d_occ; P.nproc = d_nproc; P.wnbytes = d_wnb; P.idle = d_idle;
  P.sat = d_sat; P.total_occ = total_occ; P.total_nthreads = total_nthreads; P.bw = bandwidth; P.T = T;
  P.victim = d_victim; P.duration = d_dur; P.fast = d_fast; P.dep_ptr = d_dep_ptr; P.dep_idx = d_dep_idx;
  P.d_nbytes = d_dnb; P.d_get_nbytes = d_dgnb; P.h_ptr = d_h_ptr; P.h_idx = d_h_idx; P.key_sorted = C.keys_sorted;
  C.P = P;
  C.W = W;
  C.T = T;
  C.NK = NK;
  int bits = 1;
  while ((1ll << bits) < NK) bits++;
  int rc = 0;
  int32_t nst = 0;
  if (T > 0) {
    rc = timed_launch(e, 4, [&] {
      hipLaunchKernelGGL(S::k_steal_levels, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, s, P);
      int32_t* key_in = P.key;
      if (ordered) {
        // ascending (priority, arrival): arrival first, then priority, both stable; the bin
        // sort below then keeps that order inside each bin. Keys go through the sign bit
        // flipped (int64 order as uint64).
        const unsigned gt = (unsigned)((T + 255) / 256);
        chk(hipMemcpyAsync(d_ok1, C.order_prio.data(), T * 8, hipMemcpyHostToDevice, s));
        chk(hipMemcpyAsync(d_ok2, C.order_arr.data(), T * 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(S::k_flip_sign, dim3(gt), dim3(256), 0, s, d_ok1, T);
        hipLaunchKernelGGL(S::k_flip_sign, dim3(gt), dim3(256), 0, s, d_ok2, T);
        hipLaunchKernelGGL(dgp::k_iota32, dim3(gt), dim3(256), 0, s, d_perm1, (int)T);
        size_t tb = tmp_bytes;
        chk(hipcub::DeviceRadixSort::SortPairs(C.d_tmp, tb, d_ok2, d_ok3, d_perm1, d_perm2, Tn, 0, 64, s));
        hipLaunchKernelGGL(S::k_gather_u64, dim3(gt), dim3(256), 0, s, d_ok1, d_perm2, d_ok3, T);
        tb = tmp_bytes;
        chk(hipcub::DeviceRadixSort::SortPairs(C.d_tmp, tb, d_ok3, d_ok2, d_perm2, C.d_vals, Tn, 0, 64, s));
        hipLaunchKernelGGL(S::k_gather_i32, dim3(gt), dim3(256), 0, s, P.key, C.d_vals, d_perm1, T);
        key_in = d_perm1;  // the bin keys in that order, the task ids (C.d_vals) beside them
      } else {
        hipLaunchKernelGGL(dgp::k_iota32, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, s, C.d_vals, (int)T);
      }
      size_t tb = tmp_bytes;
      chk(hipcub::DeviceRadixSort::SortPairs(C.d_tmp, tb, key_in, C.keys_sorted, C.d_vals, P.order, Tn, 0, bits, s));
      tb = tmp_bytes;
      chk(hipcub::DeviceScan::ExclusiveSum(C.d_tmp, tb, P.bin_cnt, P.bin_ptr, NK, s));
    });
    if (!rc) rc = timed_launch(e, 5, [&] {
      // initial thieves in (stack time, ws.nbytes, index) order: two stable radix sorts
      const unsigned gw = (unsigned)((W + 255) / 256);
      hipLaunchKernelGGL(S::k_thief_keys, dim3(gw), dim3(256), 0, s, P);
      size_t tb = tmp_bytes;
      chk(hipcub::DeviceRadixSort::SortPairs(C.d_tmp, tb, P.tk_nb, P.tk_nb2, P.tk_w, P.tk_w2, W, 0, 64, s));
      hipLaunchKernelGGL(S::k_gather_a, dim3(gw), dim3(256), 0, s, P);
      tb = tmp_bytes;
      chk(hipcub::DeviceRadixSort::SortPairs(C.d_tmp, tb, P.tk_a2, P.tk_a, P.tk_w2, P.th_order, W, 0, 64, s));
      hipLaunchKernelGGL(S::k_runs, dim3(1), dim3(64), 0, s, P);
    });
    if (!rc) chk(hipMemcpyAsync(&nst, P.bin_ptr + NK - 1, 4, hipMemcpyDeviceToHost, s));
  } else {
    chk(hipMemsetAsync(P.bin_ptr, 0, NK * 4, s));
    chk(hipMemsetAsync(P.n_runs, 0, 4, s));  // no thief runs are read without tasks
  }
  chk(hipStreamSynchronize(s));
  if (rc) return rc;
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("dgp_steal_load: ") + hipGetErrorString(st));
  if (nst < 0 || nst > T) return fail(e, DGP_E_STATE, "dgp_steal_load: bin scan out of range");
  C.n_stealable = nst;
  C.loaded = true;
  C.order_prio.clear();
  C.order_arr.clear();
  *n_stealable = nst;
  return 0;
}

int dgp_steal_order(dgp_engine* e, int64_t n_tasks, const int64_t* priority, const int64_t* arrival) {
  if (!e) return DGP_E_ARG;
  if (n_tasks < 0 || (n_tasks && (!priority || !arrival))) return fail(e, DGP_E_ARG, "dgp_steal_order: bad arrays");
  e->steal.order_prio.assign(priority, priority + n_tasks);
  e->steal.order_arr.assign(arrival, arrival + n_tasks);
  return 0;
}

int dgp_steal_thief_rows(dgp_engine* e, int64_t lo, int64_t hi) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e) return DGP_E_ARG;
  StealCtx& C = e->steal;
  if (!C.loaded) return fail(e, DGP_E_STATE, "dgp_steal_thief_rows: no dgp_steal_load");
  if (lo < 0 || hi < lo || hi > C.n_stealable) return fail(e, DGP_E_ARG, "dgp_steal_thief_rows: range");
  if (hi == lo) return 0;
  HIPCHK(e, hipSetDevice(e->device));
  const dgp::steal::Prob P = C.P;
  return timed_launch(e, 5, [&] {
    hipLaunchKernelGGL(dgp::steal::k_best_thief, dim3((unsigned)(((hi - lo) * 64 + 255) / 256)), dim3(256), 0,
                       e->stream, P, lo, hi);
  });
}

int64_t dgp_steal_row_bytes(void) { return (int64_t)sizeof(dgp::steal::Row); }

int dgp_steal_pack_rows(dgp_engine* e, int64_t lo, int64_t hi, void* dst) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e) return DGP_E_ARG;
  StealCtx& C = e->steal;
  if (!C.loaded) return fail(e, DGP_E_STATE, "dgp_steal_pack_rows: no dgp_steal_load");
  if (lo < 0 || hi < lo || hi > C.n_stealable || (hi > lo && !dst)) return fail(e, DGP_E_ARG, "dgp_steal_pack_rows: range");
  if (hi == lo) return 0;
  HIPCHK(e, hipSetDevice(e->device));
  hipLaunchKernelGGL(dgp::steal::k_pack_rows, dim3((unsigned)((hi - lo + 255) / 256)), dim3(256), 0, e->stream, C.P,
                     lo, hi, (dgp::steal::Row*)dst);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipStreamSynchronize(e->stream));  // the caller's collective runs on its own stream
  return 0;
}

int dgp_steal_unpack_rows(dgp_engine* e, int64_t lo, int64_t hi, const void* src) {
  if (int rc_ = resident_stop(e)) return rc_;
  if (!e) return DGP_E_ARG;
  StealCtx& C = e->steal;
  if (!C.loaded) return fail(e, DGP_E_STATE, "dgp_steal_unpack_rows: no dgp_steal_load");
  if (lo < 0 || hi < lo || hi > C.n_stealable || (hi > lo && !src))
    return fail(e, DGP_E_ARG, "dgp_steal_unpack_rows: range");
  if (hi == lo) return 0;
  HIPCHK(e, hipSetDevice(e->device));
  hipLaunchKernelGGL(dgp::steal::k_unpack_rows, dim3((unsigned)((hi - lo + 255) / 256)), dim3(256), 0, e->stream,
                     C.P, lo, hi, (const dgp::steal::Row*)src);
  HIPCHK(e, hipGetLastError());
  return 0;
}

int dgp_steal_run(dgp_engine* e, int8_t* level_out, int32_t* st_task, int32_t* st_victim, int32_t* st_thief,
                  int32_t* st_level, double* st_cost, double* st_occ_victim, double* st_occ_thief, int64_t* n_steals,
                  double* inflight_occ, int32_t* inflight_tasks, uint8_t* idle_out, uint8_t* sat_out,
                  uint8_t* checked_out) {
  if (int rc_ = resident_stop(e)) return rc_;
  namespace S = dgp::steal;
  if (!e) return DGP_E_ARG;
  StealCtx& C = e->steal;
  if (!C.loaded) return fail(e, DGP_E_STATE, "dgp_steal_run: no dgp_steal_load");
  if (!n_steals || !inflight_occ || !inflight_tasks || !idle_out || !sat_out)
    return fail(e, DGP_E_ARG, "dgp_steal_run: null pointers");
  HIPCHK(e, hipSetDevice(e->device));
  hipStream_t s = e->stream;
  const S::Prob P = C.P;
  const int64_t T = C.T;
  const int32_t W = C.W;
  int rc = timed_launch(e, 6, [&] {
    hipLaunchKernelGGL(S::k_balance, dim3(1), dim3(64), S::balance_lds_bytes(W), s, P);
  });
  if (rc) return rc;
  hipError_t st = hipSuccess;
  auto chk = [&](hipError_t x) {
    if (x != hipSuccess && st == hipSuccess) st = x;
  };
  long long ns = 0;
  chk(hipMemcpyAsync(&ns, P.n_steals, 8, hipMemcpyDeviceToHost, s));
  chk(hipStreamSynchronize(s));
  if (st == hipSuccess) {
    *n_steals = ns;
    auto d2h = [&](void* dst, const void* src, size_t bytes) {
      if (dst && bytes) chk(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    };
    d2h(level_out, P.level, T);
    d2h(st_task, P.st_task, ns * 4); d2h(st_victim, P.st_victim, ns * 4); d2h(st_thief, P.st_thief, ns * 4);
    d2h(st_level, P.st_level, ns * 4); d2h(st_cost, P.st_cost, ns * 8); d2h(st_occ_victim, P.st_occ_victim, ns * 8);
    d2h(st_occ_thief, P.st_occ_thief, ns * 8);
    d2h(inflight_occ, P.inflight_occ, W * 8); d2h(inflight_tasks, P.inflight_tasks, W * 4);
    d2h(idle_out, P.idle_out, W); d2h(sat_out, P.sat_out, W); d2h(checked_out, P.checked, W);
    chk(hipStreamSynchronize(s));
  }
  if (st != hipSuccess) return fail(e, DGP_E_HIP, std::string("dgp_steal_run: ") + hipGetErrorString(st));
  return 0;
}

int dgp_steal_balance(dgp_engine* e, int32_t W, const int32_t* nthreads, const double* occ, const int32_t* nproc,
                      const int64_t* wnbytes, const uint8_t* idle, const uint8_t* sat, double total_occ,
                      int64_t total_nthreads, int64_t bandwidth, int64_t T, const int32_t* victim,
                      const double* duration, const uint8_t* fast, const int64_t* dep_ptr, const int32_t* dep_idx,
                      int64_t n_data, const int64_t* d_nbytes, const int64_t* d_get_nbytes, const int64_t* h_ptr,
                      const int32_t* h_idx, const int64_t* r_ptr, const int32_t* r_idx, const uint8_t* r_flags,
                      const int8_t* level_in, const double* ifo_in, const int32_t* ift_in,
                      int8_t* level_out, int32_t* st_task, int32_t* st_victim,
                      int32_t* st_thief, int32_t* st_level, double* st_cost, double* st_occ_victim,
                      double* st_occ_thief, int64_t* n_steals, double* inflight_occ, int32_t* inflight_tasks,
                      uint8_t* idle_out, uint8_t* sat_out, uint8_t* checked_out) {
  if (int rc_ = resident_stop(e)) return rc_;
  int64_t n = 0;
  if (int rc = dgp_steal_load(e, W, nthreads, occ, nproc, wnbytes, idle, sat, total_occ, total_nthreads, bandwidth, T,
                              victim, duration, fast, dep_ptr, dep_idx, n_data, d_nbytes, d_get_nbytes, h_ptr, h_idx,
                              r_ptr, r_idx, r_flags, level_in, ifo_in, ift_in, &n))
    return rc;
  if (int rc = dgp_steal_thief_rows(e, 0, n)) return rc;
  return dgp_steal_run(e, level_out, st_task, st_victim, st_thief, st_level, st_cost, st_occ_victim, st_occ_thief,
                       n_steals, inflight_occ, inflight_tasks, idle_out, sat_out, checked_out);
}

}  // extern "C"
