// ORACLE — test infrastructure, not product code.
//
// CPU restatement of the reference scheduler's placement hot path, replayed in the
// golden-vector wave order (tests/golden/gen_golden.py). Only tests/, smoke() and
// bench.py's cpu_baseline leg may load it (ctypes, via oracle/oracle.py); the HIP
// engine in distributed_amd/ never calls it.
//
// Pinned against tests/golden/*.npz, which were produced by the reference
// SchedulerState itself (tests/test_oracle_golden.py checks every placement
// bit-for-bit and every per-round worker snapshot).
//
// Every function below names the reference code it restates
// (/root/reference/distributed/scheduler.py unless stated otherwise).
// Deliberate representation changes (same observable behaviour in the replay):
//  * TaskState.waiting_on / waiters are counts, not sets (they are only ever
//    discarded from, each member once, in this replay).
//  * Set iteration that decides ties uses the canonical order of gen_golden.py:
//    ascending worker index (worker_objective gets the index as last key).
//  * SortedDict `idle` is an index-ordered membership bitmap + Fenwick tree.
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off; no FMA, same rounding as CPython).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <queue>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <iterator>
#include <utility>
#include <vector>

extern "C" {
struct orc_graph {
  int64_t n_tasks, n_workers, n_prefixes, n_groups;
  const int64_t* dep_ptr;
  const int32_t* dep_idx;
  const int64_t* prio;
  const int32_t* prefix_id;
  const int32_t* group_id;
  const uint8_t* wanted;
  const int8_t* rootish_override;
  const int64_t* nbytes;
  const double* start;
  const double* stop;
  const int32_t* nthreads;
  const int32_t* group_prefix;
  const double* prefix_default_dur;
  int64_t bandwidth;
  int64_t default_data_size;
  double unknown_duration;
  double saturation;  // +inf allowed
  // worker restrictions (optional, all null = none): valid_workers(ts) (:3043-3107)
  // resolved to worker indices (CSR, ascending), and flags bit 0 = the task has
  // restrictions (a non-empty restriction set; its valid set may still be empty),
  // bit 1 = loose_restrictions (:8584-8586)
  const int64_t* restr_ptr;
  const int32_t* restr_idx;
  const uint8_t* restr_flags;
  // workers joining mid-replay (optional, n_joins = 0: none): join k happens before the
  // join_before[k]-th completion (0-based, completions counted in replay order), with
  // join_nthreads[k] threads and the next worker index (Scheduler.add_worker :4308-4441)
  int64_t n_joins;
  const int64_t* join_before;
  const int32_t* join_nthreads;
  // a later graph submitted mid-replay (optional): its tasks get indices n_tasks.., its
  // dependencies are relative to it (independent of this graph), priorities follow this
  // graph's, prefix / group ids over the grown tables (n_prefixes / n_groups = the totals;
  // prefix_default_dur read for the new prefixes). Submitted before the next_before-th
  // completion (Scheduler.update_graph :4662-4751 -> _create_taskstate_from_graph :4512-4653)
  const struct orc_graph* next;
  int64_t next_before;
};

struct orc_result {
  // per placement, capacity >= n_tasks
  int32_t* pl_task;
  int32_t* pl_worker;
  int64_t* pl_comm;
  double* pl_start;
  int64_t* pl_wsnbytes;
  int8_t* pl_route;
  int64_t n_placements;
  // per round, capacity max_rounds (snapshot arrays [max_rounds][W]; may be NULL)
  int64_t max_rounds;
  int64_t snap_stride;  // workers per snapshot row (>= n_workers + n_joins; 0: n_workers)
  int64_t n_rounds;
  int32_t* round_nplaced;
  double* round_occ;
  int64_t* round_wnbytes;
  int32_t* round_nproc;
  uint8_t* round_idle;
  uint8_t* round_sat;
  uint8_t* round_itc;
  int32_t* round_nqueued;
  uint8_t* final_state;  // n_tasks (may be NULL)
  double seconds;        // wall time of the replay (graph build excluded)
  char error[256];
};
}

namespace {

enum TState : uint8_t { RELEASED = 0, WAITING, PROCESSING, QUEUED, NO_WORKER, MEMORY, ERRED, FORGOTTEN };
enum Route : int8_t { R_NONROOTISH = 0, R_ROOTISH_Q = 1, R_ROOTISH_NOQ = 2, R_FASTPATH = 3 };

struct Fail : std::runtime_error {
  using std::runtime_error::runtime_error;
};
#define ORC_CHECK(c, msg) \
  do {                    \
    if (!(c)) throw Fail(msg); \
  } while (0)

// insertion-ordered {prefix: count} dict with delete-on-zero
// (WorkerState.task_prefix_count defaultdict, :733-784; SchedulerState._task_prefix_count_global)
struct PrefixCounts {
  std::vector<std::pair<int32_t, int64_t>> items;
  void inc(int32_t p) {
    for (auto& it : items)
      if (it.first == p) { it.second++; return; }
    items.emplace_back(p, 1);
  }
  void dec(int32_t p) {
    for (size_t i = 0; i < items.size(); i++)
      if (items[i].first == p) {
        if (--items[i].second == 0) items.erase(items.begin() + i);
        return;
      }
    throw Fail("prefix count underflow");
  }
};

struct Fenwick {  // order-statistics over worker indices (SortedDict keyed by address)
  std::vector<int32_t> t;
  int n = 0, cnt = 0;
  void init(int n_) { n = n_; t.assign(n + 1, 0); cnt = 0; }
  void add(int i, int v) {
    cnt += v;
    for (i++; i <= n; i += i & -i) t[i] += v;
  }
  int kth(int k) const {  // 0-based k-th member
    int pos = 0, logn = 1;
    while ((logn << 1) <= n) logn <<= 1;
    for (int step = logn; step; step >>= 1)
      if (pos + step <= n && t[pos + step] <= k) { pos += step; k -= t[pos]; }
    return pos;
  }
};

struct Worker {
  int32_t nthreads = 1;
  int64_t nproc = 0;         // len(processing)
  int64_t nlong = 0;         // len(long_running)
  PrefixCounts prefix;       // task_prefix_count
  std::unordered_map<int32_t, int32_t> needs;  // needs_what
  int64_t net_occ = 0;       // _network_occ (int)
  int64_t nbytes = 0;        // nbytes
  uint8_t idle = 0, saturated = 0, itc = 0;
  int32_t slot_cap = 0;      // max(ceil(sat * nthreads), 1)
};

struct Group {
  int64_t size = 0;
  int64_t n_released = 0, n_waiting = 0;
  int32_t last_worker = -1;
  int64_t last_worker_tasks_left = 0;
  int8_t rootish_static = 0;
};

struct Prefix {
  double duration_average = -1;
  double max_exec_time = -1;
};

struct Recs {  // ordered dict {task: finish} with popitem() LIFO and update() keeping positions
  std::vector<std::pair<int32_t, uint8_t>> items;
};

// the graph as the replay holds it: owned copies, so that a later graph can be appended
struct GraphArrays {
  std::vector<int64_t> dep_ptr, prio, nbytes;
  std::vector<int32_t> dep_idx, prefix_id, group_id;
  std::vector<uint8_t> wanted;
  std::vector<int8_t> rootish_override;
  std::vector<double> start, stop, prefix_default_dur;
  int64_t n_prefixes = 0, n_groups = 0;
  // append graph h (dependencies relative to it) after n0 tasks
  void append(const orc_graph& h, int64_t n0) {
    const int64_t n = h.n_tasks, e0 = dep_ptr.empty() ? 0 : dep_ptr.back();
    if (dep_ptr.empty()) dep_ptr.push_back(0);
    for (int64_t t = 0; t < n; t++) {
      dep_ptr.push_back(e0 + h.dep_ptr[t + 1]);
      prio.push_back(h.prio[t]);
      nbytes.push_back(h.nbytes[t]);
      prefix_id.push_back(h.prefix_id[t]);
      group_id.push_back(h.group_id[t]);
      wanted.push_back(h.wanted[t]);
      rootish_override.push_back(h.rootish_override[t]);
      start.push_back(h.start[t]);
      stop.push_back(h.stop[t]);
    }
    for (int64_t k = 0; k < h.dep_ptr[n]; k++) dep_idx.push_back((int32_t)(h.dep_idx[k] + n0));
    for (int64_t q = n_prefixes; q < h.n_prefixes; q++) prefix_default_dur.push_back(h.prefix_default_dur[q]);
    n_prefixes = std::max(n_prefixes, h.n_prefixes);
    n_groups = std::max(n_groups, h.n_groups);
  }
};

struct Replay {
  const orc_graph& g;
  orc_result& r;
  GraphArrays G;
  int64_t N, W;
  std::vector<int64_t> dpt_ptr;
  std::vector<int32_t> dpt_idx;
  std::vector<uint8_t> state;
  std::vector<int32_t> waiting_on;  // |waiting_on|
  std::vector<int32_t> waiters;     // |waiters|
  std::vector<int32_t> processing_on;
  std::vector<int64_t> cur_nbytes;
  std::vector<std::vector<int32_t>> who_has;
  std::vector<int64_t> run_id;
  std::vector<uint8_t> in_queue;
  std::vector<Worker> ws;
  std::vector<Group> groups;
  std::vector<Prefix> prefixes;
  PrefixCounts prefix_global;
  double net_occ_global = 0.0;
  int64_t total_nthreads = 0;
  int64_t n_tasks_counter = 0;
  int64_t run_id_counter = 0;
  Fenwick idle;
  int64_t n_saturated = 0, n_itc = 0;
  using QItem = std::pair<int64_t, int64_t>;  // (priority rank, insertion counter) -> task via map
  std::priority_queue<std::tuple<int64_t, int64_t, int32_t>, std::vector<std::tuple<int64_t, int64_t, int32_t>>,
                      std::greater<>>
      queue;
  int64_t queue_inc = 0, queue_len = 0;
  int64_t n_unrunnable = 0;
  bool sat_inf;
  // recommendations scratch: position of a key inside the active Recs, -1 if absent
  std::vector<int32_t> rec_pos;

  Replay(const orc_graph& g_, orc_result& r_) : g(g_), r(r_), N(g_.n_tasks), W(g_.n_workers) {
    G.append(g, 0);
    sat_inf = std::isinf(g.saturation);
    build_dependents();
    state.assign(N, RELEASED);
    waiting_on.assign(N, 0);
    waiters.assign(N, 0);
    processing_on.assign(N, -1);
    cur_nbytes.assign(N, -1);
    who_has.assign(N, {});
    run_id.assign(N, -1);
    in_queue.assign(N, 0);
    rec_pos.assign(N, -1);
    ws.resize(W);
    for (int64_t w = 0; w < W; w++) {
      ws[w].nthreads = g.nthreads[w];
      total_nthreads += g.nthreads[w];
      if (!sat_inf) ws[w].slot_cap = std::max((int32_t)std::ceil(g.saturation * ws[w].nthreads), (int32_t)1);
    }
    prefixes.resize(G.n_prefixes);
    for (int64_t p = 0; p < G.n_prefixes; p++) prefixes[p].duration_average = G.prefix_default_dur[p];
    groups.resize(G.n_groups);
    for (int64_t t = 0; t < N; t++) {
      groups[G.group_id[t]].size++;
      groups[G.group_id[t]].n_released++;
    }
    // TaskGroup.dependencies (:1474) -> is_rootish inputs (:2929-2947); total_nthreads is
    // constant during a replay, so the heuristic is static per group.
    build_group_deps();
    rootish_groups();
    idle.init((int)(W + g.n_joins));  // room for the workers that join (index order = address order)
  }
  void build_dependents() {  // TaskState.dependents (:1220), over the whole graph
    std::vector<int64_t> deg(N + 1, 0);
    for (int64_t t = 0; t < N; t++)
      for (int64_t k = G.dep_ptr[t]; k < G.dep_ptr[t + 1]; k++) deg[G.dep_idx[k] + 1]++;
    dpt_ptr.assign(N + 1, 0);
    for (int64_t t = 0; t < N; t++) dpt_ptr[t + 1] = dpt_ptr[t] + deg[t + 1];
    dpt_idx.resize(dpt_ptr[N]);
    std::vector<int64_t> fill(dpt_ptr.begin(), dpt_ptr.end() - 1);
    for (int64_t t = 0; t < N; t++)
      for (int64_t k = G.dep_ptr[t]; k < G.dep_ptr[t + 1]; k++) dpt_idx[fill[G.dep_idx[k]]++] = (int32_t)t;
  }
  void build_group_deps() {  // TaskGroup.dependencies (:1474)
    gdeps.assign(G.n_groups, {});
    for (int64_t t = 0; t < N; t++)
      for (int64_t k = G.dep_ptr[t]; k < G.dep_ptr[t + 1]; k++) gdeps[G.group_id[t]].push_back(G.group_id[G.dep_idx[k]]);
    for (int64_t gi = 0; gi < G.n_groups; gi++) {
      auto& v = gdeps[gi];
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
    }
  }
  std::vector<std::vector<int32_t>> gdeps;  // TaskGroup.dependencies
  void rootish_groups() {  // is_rootish's group part (:2941-2947) for the current total_nthreads
    for (int64_t gi = 0; gi < G.n_groups; gi++) {
      int64_t sum_len = 0;
      for (int32_t d : gdeps[gi]) sum_len += groups[d].size;
      groups[gi].rootish_static =
          (groups[gi].size > total_nthreads * 2 && (int64_t)gdeps[gi].size() < 5 && sum_len < 5) ? 1 : 0;
    }
  }
  // Scheduler.add_worker (:4308-4441), the placement part: the WorkerState joins workers /
  // running with the next index, total_nthreads grows (:4383), check_idle_saturated(ws)
  // (:4398), bulk_schedule_unrunnable_after_adding_worker (:3173-3186, nothing when no task
  // is no-worker) and stimulus_queue_slots_maybe_opened (:4416-4420)
  // a later, independent graph: TaskStates appended (TaskPrefix / TaskGroup shared by name
  // through the ids), group sizes and is_rootish's group part over the grown graph, then
  // every new task recommended "waiting" in descending priority (:4600-4651)
  void add_graph(const orc_graph& h) {
    // the earlier graph may carry restrictions (its rows stay); the later graph has none
    ORC_CHECK(!h.restr_flags, "a later graph with restrictions: not in the replay subset");
    const int64_t n0 = N, n1 = N + h.n_tasks;
    G.append(h, n0);
    N = n1;
    state.resize(n1, RELEASED);
    waiting_on.resize(n1, 0);
    waiters.resize(n1, 0);
    processing_on.resize(n1, -1);
    cur_nbytes.resize(n1, -1);
    who_has.resize(n1);
    run_id.resize(n1, -1);
    in_queue.resize(n1, 0);
    rec_pos.resize(n1, -1);
    build_dependents();
    for (int64_t p = (int64_t)prefixes.size(); p < G.n_prefixes; p++) {
      prefixes.emplace_back();
      prefixes.back().duration_average = G.prefix_default_dur[p];
    }
    groups.resize(G.n_groups);
    for (int64_t t = n0; t < n1; t++) {
      groups[G.group_id[t]].size++;
      groups[G.group_id[t]].n_released++;
    }
    build_group_deps();
    rootish_groups();
    std::vector<int32_t> order;
    for (int64_t t = n0; t < n1; t++) order.push_back((int32_t)t);
    std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return G.prio[a] > G.prio[b]; });
    Recs rc;
    for (int32_t t : order) rc.items.emplace_back(t, WAITING);
    transitions(std::move(rc));
  }

  void add_worker(int32_t nthreads) {
    ORC_CHECK(n_unrunnable == 0, "worker join with no-worker tasks: not in the replay subset");
    Worker x;
    x.nthreads = nthreads;
    if (!sat_inf) x.slot_cap = std::max((int32_t)std::ceil(g.saturation * nthreads), (int32_t)1);
    ws.push_back(x);
    W++;
    total_nthreads += nthreads;
    rootish_groups();
    check_idle_saturated((int32_t)(W - 1));
    queue_slots_maybe_opened();
  }

  // ---------------------------------------------------------------- helpers
  int64_t get_nbytes(int32_t t) const {  // TaskState.get_nbytes :1477-1478
    return cur_nbytes[t] >= 0 ? cur_nbytes[t] : g.default_data_size;
  }
  bool holds(int32_t t, int32_t w) const {
    for (int32_t x : who_has[t])
      if (x == w) return true;
    return false;
  }
  void set_state(int32_t t, uint8_t s) {  // TaskState.state setter :1464-1469 (group counts)
    Group& gr = groups[G.group_id[t]];
    if (state[t] == RELEASED) gr.n_released--;
    if (state[t] == WAITING) gr.n_waiting--;
    if (s == RELEASED) gr.n_released++;
    if (s == WAITING) gr.n_waiting++;
    state[t] = s;
  }
  double prefix_duration(int32_t p) const {  // _calc_occupancy :1892-1899
    double d = prefixes[p].duration_average;
    if (d < 0) {
      if (prefixes[p].max_exec_time > 0)
        d = 2 * prefixes[p].max_exec_time;
      else
        d = g.unknown_duration;
    }
    return d;
  }
  double calc_occupancy(const PrefixCounts& pc, double network_occ) const {  // :1884-1903
    double res = 0.0;
    for (auto& it : pc.items) res += prefix_duration(it.first) * (double)it.second;
    return res + network_occ / (double)g.bandwidth;
  }
  double occupancy(int32_t w) const {  // WorkerState.occupancy :840-844
    return calc_occupancy(ws[w].prefix, (double)ws[w].net_occ);
  }
  double total_occupancy() const { return calc_occupancy(prefix_global, net_occ_global); }  // :1877

  // restrictions are rows of the first graph (a later graph's tasks have none)
  bool restricted(int32_t t) const { return g.restr_flags && t < g.n_tasks && (g.restr_flags[t] & 1); }
  bool loose(int32_t t) const { return g.restr_flags && t < g.n_tasks && (g.restr_flags[t] & 2); }

  bool is_rootish(int32_t t) const {  // :2929-2947
    int8_t ov = G.rootish_override[t];
    if (ov >= 0) return ov != 0;
    if (restricted(t)) return false;  // :2939-2940
    return groups[G.group_id[t]].rootish_static != 0;
  }

  int64_t task_slots_available(int32_t w) const {  // _task_slots_available :8762-8767
    return (int64_t)ws[w].slot_cap - (ws[w].nproc - ws[w].nlong);
  }
  bool worker_full(int32_t w) const {  // _worker_full :8770-8773
    if (sat_inf) return false;
    return task_slots_available(w) <= 0;
  }

  bool is_unoccupied(int32_t w, double occ, int64_t p) const {  // :2997-3004
    int64_t nt = ws[w].nthreads;
    return p < nt || occ < (double)nt * (total_occupancy() / (double)total_nthreads) / 2;
  }

  void check_idle_saturated(int32_t w, double occ = -1.0) {  // :2949-2995
    if (total_nthreads == 0) return;
    if (occ < 0) occ = occupancy(w);
    Worker& x = ws[w];
    int64_t p = x.nproc;
    if (x.saturated) { x.saturated = 0; n_saturated--; }
    if (is_unoccupied(w, occ, p)) {
      if (!x.idle) { x.idle = 1; idle.add(w, 1); }
    } else {
      if (x.idle) { x.idle = 0; idle.add(w, -1); }
      int64_t nc = x.nthreads;
      if (p > nc) {
        double pending = occ * (double)(p - nc) / (double)(p * nc);
        if (0.4 < pending && pending > 1.9 * (total_occupancy() / (double)total_nthreads)) {
          x.saturated = 1;
          n_saturated++;
        }
      }
    }
    bool want = !worker_full(w);
    if (want && !x.itc) { x.itc = 1; n_itc++; }
    if (!want && x.itc) { x.itc = 0; n_itc--; }
  }

  // worker_objective :3131-3146 (+ canonical worker-index tie-break)
  struct Obj {
    double start;
    int64_t nbytes;
    int32_t w;
    int64_t comm;
    bool operator<(const Obj& o) const {
      if (start != o.start) return start < o.start;
      if (nbytes != o.nbytes) return nbytes < o.nbytes;
      return w < o.w;
    }
  };
  Obj worker_objective(int32_t t, int32_t w) const {
    int64_t comm = 0;
    for (int64_t k = G.dep_ptr[t]; k < G.dep_ptr[t + 1]; k++) {
      int32_t d = G.dep_idx[k];
      if (!holds(d, w)) comm += get_nbytes(d);
    }
    double stack_time = occupancy(w) / (double)ws[w].nthreads;
    double start_time = stack_time + (double)comm / (double)g.bandwidth;
    return Obj{start_time, ws[w].nbytes, w, comm};
  }

  // ----------------------------------------------------------- decide_worker*
  int32_t decide_worker_rootish_queuing_enabled() {  // :2195-2245
    if (n_itc == 0) return -1;
    int32_t best = -1;
    double bkey = 0;
    for (int32_t w = 0; w < W; w++) {  // min over idle_task_count, first minimum in index order
      if (!ws[w].itc) continue;
      double key = (double)ws[w].nproc / (double)ws[w].nthreads;
      if (best < 0 || key < bkey) { best = w; bkey = key; }
    }
    return best;
  }

  int32_t decide_worker_rootish_queuing_disabled(int32_t t) {  // :2135-2193
    // pool = self.idle.values() if self.idle else self.running  (all workers run here)
    bool use_idle = idle.cnt > 0;
    Group& tg = groups[G.group_id[t]];
    int32_t w;
    if (tg.last_worker >= 0 && tg.last_worker_tasks_left) {
      w = tg.last_worker;
    } else {
      Obj best{};
      bool have = false;
      for (int32_t c = 0; c < W; c++) {
        if (use_idle && !ws[c].idle) continue;
        Obj o = worker_objective(t, c);
        if (!have || o < best) { best = o; have = true; }
      }
      if (!have) return -1;
      w = best.w;
      tg.last_worker_tasks_left =
          (int64_t)std::floor(((double)tg.size / (double)total_nthreads) * (double)ws[w].nthreads);
    }
    tg.last_worker = (tg.n_released + tg.n_waiting > 1) ? w : -1;
    tg.last_worker_tasks_left -= 1;
    return w;
  }

  // module-level decide_worker :8550-8593; valid = valid_workers(ts) or null (None)
  int32_t decide_worker(int32_t t, const std::vector<int32_t>* valid = nullptr) {
    std::vector<int32_t> cand;
    for (int64_t k = G.dep_ptr[t]; k < G.dep_ptr[t + 1]; k++)
      for (int32_t w : who_has[G.dep_idx[k]]) cand.push_back(w);
    std::sort(cand.begin(), cand.end());
    cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
    if (!valid) {
      if (cand.empty()) {  // candidates = all_workers.copy()
        cand.resize(W);
        for (int32_t w = 0; w < W; w++) cand[w] = w;
      }
    } else {  // candidates &= valid_workers; else valid_workers; else the loose retry
      std::vector<int32_t> both;
      std::set_intersection(cand.begin(), cand.end(), valid->begin(), valid->end(), std::back_inserter(both));
      cand.swap(both);
      if (cand.empty()) {
        cand = *valid;
        if (cand.empty() && loose(t)) return decide_worker(t, nullptr);
      }
    }
    if (cand.empty()) return -1;
    if (cand.size() == 1) return cand[0];
    Obj best = worker_objective(t, cand[0]);
    for (size_t i = 1; i < cand.size(); i++) {
      Obj o = worker_objective(t, cand[i]);
      if (o < best) best = o;
    }
    return best.w;
  }

  int32_t decide_worker_non_rootish(int32_t t, Route& route) {  // :2247-2311
    if (W == 0) return -1;
    if (restricted(t)) {  // valid_workers(ts) is not None (every worker runs here)
      route = R_NONROOTISH;
      std::vector<int32_t> valid(g.restr_idx + g.restr_ptr[t], g.restr_idx + g.restr_ptr[t + 1]);
      return decide_worker(t, &valid);
    }
    if (G.dep_ptr[t + 1] > G.dep_ptr[t]) {
      route = R_NONROOTISH;
      return decide_worker(t);
    }
    route = R_FASTPATH;
    // worker_pool = self.idle or self.workers (both ordered by address = index)
    bool use_idle = idle.cnt > 0;
    int64_t n = use_idle ? idle.cnt : W;
    auto pool_at = [&](int64_t i) -> int32_t { return use_idle ? idle.kth((int)i) : (int32_t)i; };
    if (n < 20) {
      int32_t best = pool_at(0);
      double bocc = occupancy(best);
      for (int64_t i = 1; i < n; i++) {
        int32_t c = pool_at(i);
        double o = occupancy(c);
        if (o < bocc) { best = c; bocc = o; }
      }
      if (bocc == 0) {
        int64_t start = n_tasks_counter % n;
        for (int64_t i = 0; i < n; i++) {
          int32_t c = pool_at((i + start) % n);
          if (occupancy(c) == 0) { best = c; break; }
        }
      }
      return best;
    }
    return pool_at(n_tasks_counter % n);
  }

  // ------------------------------------------------------------ placement commit
  void inc_needs_replica(int32_t w, int32_t d) {  // :800-813
    auto it = ws[w].needs.find(d);
    if (it == ws[w].needs.end()) {
      ws[w].needs.emplace(d, 1);
      int64_t nb = get_nbytes(d);
      ws[w].net_occ += nb;
      net_occ_global += (double)nb;
    } else {
      it->second++;
    }
  }
  void dec_needs_replica(int32_t w, int32_t d) {  // :815-823
    auto it = ws[w].needs.find(d);
    if (--it->second == 0) {
      ws[w].needs.erase(it);
      int64_t nb = get_nbytes(d);
      ws[w].net_occ -= nb;
      net_occ_global -= (double)nb;
    }
  }

  void add_to_processing(int32_t t, int32_t w, Route route) {  // _add_to_processing :3199-3256
    // record the parity tuple before mutating (gen_golden.py does the same)
    Obj o = worker_objective(t, w);
    int64_t i = r.n_placements++;
    r.pl_task[i] = t;
    r.pl_worker[i] = w;
    r.pl_comm[i] = o.comm;
    r.pl_start[i] = o.start;
    r.pl_wsnbytes[i] = ws[w].nbytes;
    r.pl_route[i] = route;
    // WorkerState.add_to_processing :733-745
    ws[w].prefix.inc(G.prefix_id[t]);
    prefix_global.inc(G.prefix_id[t]);
    ws[w].nproc++;
    for (int64_t k = G.dep_ptr[t]; k < G.dep_ptr[t + 1]; k++) {
      int32_t d = G.dep_idx[k];
      ORC_CHECK(!who_has[d].empty(), "dependency without replica at placement");
      if (!holds(d, w)) inc_needs_replica(w, d);
    }
    processing_on[t] = w;
    set_state(t, PROCESSING);
    check_idle_saturated(w);
    n_tasks_counter++;
    run_id[t] = run_id_counter++;  // _task_to_msg :3427
  }

  // ------------------------------------------------------------- transitions
  void rec_set(Recs& rc, int32_t t, uint8_t finish) {
    // a transition function's own return dict (insertion-ordered; keys are distinct here)
    rc.items.emplace_back(t, finish);
  }

  Recs t_released_waiting(int32_t t) {  // :2078-2119
    Recs rc;
    set_state(t, WAITING);
    int32_t wo = 0;
    for (int64_t k = G.dep_ptr[t]; k < G.dep_ptr[t + 1]; k++) {
      int32_t d = G.dep_idx[k];
      if (who_has[d].empty()) wo++;
      if (state[d] == RELEASED)
        rec_set(rc, d, WAITING);
      else
        waiters[d]++;
    }
    waiting_on[t] = wo;
    int32_t wt = 0;
    for (int64_t k = dpt_ptr[t]; k < dpt_ptr[t + 1]; k++) wt += state[dpt_idx[k]] == WAITING;
    waiters[t] = wt;
    if (wo == 0) rec_set(rc, t, PROCESSING);
    return rc;
  }

  Recs t_waiting_processing(int32_t t) {  // :2313-2336
    Recs rc;
    int32_t w;
    Route route;
    if (is_rootish(t)) {
      if (sat_inf) {
        route = R_ROOTISH_NOQ;
        if ((w = decide_worker_rootish_queuing_disabled(t)) < 0) { rec_set(rc, t, NO_WORKER); return rc; }
      } else {
        route = R_ROOTISH_Q;
        if ((w = decide_worker_rootish_queuing_enabled()) < 0) { rec_set(rc, t, QUEUED); return rc; }
      }
    } else {
      if ((w = decide_worker_non_rootish(t, route)) < 0) { rec_set(rc, t, NO_WORKER); return rc; }
    }
    add_to_processing(t, w, route);
    return rc;
  }

  Recs t_queued_processing(int32_t t) {  // :2797-2808
    int32_t w = decide_worker_rootish_queuing_enabled();
    if (w >= 0) {
      in_queue[t] = 0;  // queued.discard
      queue_len--;
      add_to_processing(t, w, R_ROOTISH_Q);
    }
    return {};
  }

  Recs t_no_worker_processing(int32_t t) {  // :2121-2133
    Route route;
    int32_t w = decide_worker_non_rootish(t, route);
    if (w >= 0) {
      n_unrunnable--;
      add_to_processing(t, w, route);
    }
    return {};
  }

  Recs t_waiting_queued(int32_t t) {  // :2761-2770
    set_state(t, QUEUED);
    in_queue[t] = 1;
    queue_len++;
    queue.emplace(G.prio[t], queue_inc++, t);
    return {};
  }

  Recs t_waiting_no_worker(int32_t t) {  // :2772-2782
    set_state(t, NO_WORKER);
    n_unrunnable++;
    return {};
  }

  Recs t_processing_memory(int32_t t, int64_t nbytes, double start, double stop) {  // :2366-2442
    int32_t w = processing_on[t];
    ORC_CHECK(w >= 0, "processing->memory without worker");
    // TaskGroup.add_duration -> TaskPrefix.add_duration :977-985 ("compute" action)
    double duration = stop - start;
    Prefix& pf = prefixes[G.prefix_id[t]];
    double old = pf.duration_average;
    if (old < 0)
      pf.duration_average = duration;
    else
      pf.duration_average = 0.5 * duration + 0.5 * old;
    // set_nbytes :1480-1488 (who_has is empty while processing)
    cur_nbytes[t] = nbytes;
    // _exit_processing_common :3258-3281 -> WorkerState.remove_from_processing :759-771
    processing_on[t] = -1;
    ws[w].prefix.dec(G.prefix_id[t]);
    prefix_global.dec(G.prefix_id[t]);
    ws[w].nproc--;
    for (int64_t k = G.dep_ptr[t]; k < G.dep_ptr[t + 1]; k++) {
      int32_t d = G.dep_idx[k];
      if (ws[w].needs.count(d)) dec_needs_replica(w, d);
    }
    check_idle_saturated(w);
    // _add_to_memory :3283-3335
    Recs rc;
    {  // add_replica :3148 -> WorkerState.add_replica :825-838
      bool had = holds(t, w);
      if (!had) {
        int64_t nb = get_nbytes(t);
        auto it = ws[w].needs.find(t);
        if (it != ws[w].needs.end()) {
          ws[w].needs.erase(it);
          ws[w].net_occ -= nb;
          net_occ_global -= (double)nb;
        }
        who_has[t].push_back(w);
        ws[w].nbytes += nb;
      }
    }
    // frontier release: dependents in descending priority
    std::vector<int32_t> deps(dpt_idx.begin() + dpt_ptr[t], dpt_idx.begin() + dpt_ptr[t + 1]);
    if (deps.size() > 1)
      std::sort(deps.begin(), deps.end(), [&](int32_t a, int32_t b) { return G.prio[a] > G.prio[b]; });
    for (int32_t x : deps) {
      if (state[x] == WAITING && waiting_on[x] > 0) {
        if (--waiting_on[x] == 0) rec_set(rc, x, PROCESSING);
      }
    }
    for (int64_t k = G.dep_ptr[t]; k < G.dep_ptr[t + 1]; k++) {
      int32_t d = G.dep_idx[k];
      if (waiters[d] > 0) waiters[d]--;
      if (waiters[d] == 0 && !G.wanted[d]) rec_set(rc, d, RELEASED);
    }
    if (waiters[t] == 0 && !G.wanted[t]) rec_set(rc, t, RELEASED);
    set_state(t, MEMORY);
    return rc;
  }

  Recs t_memory_released(int32_t t) {  // :2444-2505 + remove_all_replicas :3161-3171
    int64_t nb = get_nbytes(t);
    for (int32_t w : who_has[t]) ws[w].nbytes -= nb;
    who_has[t].clear();
    set_state(t, RELEASED);
    Recs rc;
    if (G.wanted[t] || waiters[t] > 0) rec_set(rc, t, WAITING);
    return rc;
  }

  Recs transition(int32_t t, uint8_t finish) {  // _transition :1909-2043 (table :2889-2913)
    uint8_t start = state[t];
    if (start == finish) return {};
    if (start == RELEASED && finish == WAITING) return t_released_waiting(t);
    if (start == WAITING && finish == PROCESSING) return t_waiting_processing(t);
    if (start == WAITING && finish == QUEUED) return t_waiting_queued(t);
    if (start == WAITING && finish == NO_WORKER) return t_waiting_no_worker(t);
    if (start == QUEUED && finish == PROCESSING) return t_queued_processing(t);
    if (start == NO_WORKER && finish == PROCESSING) return t_no_worker_processing(t);
    if (start == MEMORY && finish == RELEASED) return t_memory_released(t);
    char buf[128];
    snprintf(buf, sizeof buf, "transition %d -> %d of task %d not in the replay subset", start, finish, t);
    throw Fail(buf);
  }

  // _transitions :2045-2076 — popitem() is LIFO, update() keeps existing positions
  void transitions(Recs recs) {
    std::vector<std::pair<int32_t, uint8_t>>& st = recs.items;
    for (size_t i = 0; i < st.size(); i++) rec_pos[st[i].first] = (int32_t)i;
    while (!st.empty()) {
      auto [t, finish] = st.back();
      st.pop_back();
      rec_pos[t] = -1;
      Recs nr = transition(t, finish);
      for (auto& kv : nr.items) {
        int32_t p = rec_pos[kv.first];
        if (p >= 0) {
          st[p].second = kv.second;
        } else {
          rec_pos[kv.first] = (int32_t)st.size();
          st.push_back(kv);
        }
      }
    }
  }

  // Scheduler.stimulus_queue_slots_maybe_opened :4983-5023
  void queue_slots_maybe_opened() {
    if (queue_len == 0) return;
    int64_t slots = 0;
    for (int32_t w = 0; w < W; w++)
      if (ws[w].itc) slots += task_slots_available(w);
    if (slots == 0) return;
    for (int64_t k = 0; k < slots; k++) {
      if (queue_len == 0) return;
      while (!in_queue[std::get<2>(queue.top())]) queue.pop();  // HeapSet.peek
      int32_t q = std::get<2>(queue.top());
      Recs rc;
      rc.items.emplace_back(q, PROCESSING);
      transitions(rc);
    }
  }

  void snapshot(int64_t round, int64_t nplaced) {
    r.round_nplaced[round] = (int32_t)nplaced;
    if (r.round_occ) {
      const int64_t stride = r.snap_stride > 0 ? r.snap_stride : W;
      ORC_CHECK(stride >= W, "snapshot rows narrower than the worker count");
      for (int32_t w = 0; w < W; w++) {
        int64_t o = round * stride + w;
        r.round_occ[o] = occupancy(w);
        r.round_wnbytes[o] = ws[w].nbytes;
        r.round_nproc[o] = (int32_t)ws[w].nproc;
        r.round_idle[o] = ws[w].idle;
        r.round_sat[o] = ws[w].saturated;
        r.round_itc[o] = ws[w].itc;
      }
      r.round_nqueued[round] = (int32_t)queue_len;
    }
  }

  void run() {
    // Scheduler.add_worker (:4418) ends with check_idle_saturated(ws) for each worker
    for (int32_t w = 0; w < W; w++) check_idle_saturated(w);
    // update_graph (:4600-4611): every task recommended "waiting", descending priority
    std::vector<int32_t> order(N);
    for (int64_t t = 0; t < N; t++) order[t] = (int32_t)t;
    std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return G.prio[a] > G.prio[b]; });
    Recs rc;
    rc.items.reserve(N);
    for (int32_t t : order) rc.items.emplace_back(t, WAITING);
    transitions(std::move(rc));
    int64_t done = 0, round = 0, n_done = 0, k_join = 0;
    bool next_done = false;
    while (true) {
      int64_t cur = r.n_placements;
      ORC_CHECK(round < r.max_rounds, "too many rounds for the result buffers");
      snapshot(round, cur - done);
      round++;
      if (cur == done) break;
      for (int64_t i = done; i < cur; i++) {  // completions in run_id order
        while (k_join < g.n_joins && g.join_before[k_join] <= n_done) add_worker(g.join_nthreads[k_join++]);
        if (g.next && !next_done && g.next_before <= n_done) {
          next_done = true;
          add_graph(*g.next);
        }
        n_done++;
        int32_t t = r.pl_task[i];
        ORC_CHECK(state[t] == PROCESSING, "completion of a task that is not processing");
        Recs c = t_processing_memory(t, G.nbytes[t], G.start[t], G.stop[t]);
        transitions(std::move(c));
        queue_slots_maybe_opened();
      }
      done = cur;
    }
    r.n_rounds = round;
    if (r.final_state)
      for (int64_t t = 0; t < N; t++) r.final_state[t] = state[t];
  }
};

}  // namespace

extern "C" int orc_replay(const orc_graph* g, orc_result* r) {
  r->n_placements = 0;
  r->n_rounds = 0;
  r->error[0] = 0;
  try {
    Replay rp(*g, *r);
    auto t1 = std::chrono::steady_clock::now();
    rp.run();
    auto t2 = std::chrono::steady_clock::now();
    (void)t1;
    r->seconds = std::chrono::duration<double>(t2 - t1).count();
    return 0;
  } catch (const std::exception& e) {
    snprintf(r->error, sizeof r->error, "%s", e.what());
    return 1;
  }
}
