// ORACLE — test infrastructure, not product code.
//
// CPU restatement of the reference WorkStealing cost levels and one balance() call
// (/root/reference/distributed/stealing.py), the checker for the HIP balance kernel.
// Only tests/, smoke() and bench.py's cpu_baseline leg may load it (ctypes, via
// oracle/oracle.py). Pinned against tests/golden/steal_*.npz, which the reference
// WorkStealing plugin itself produced (tests/golden/gen_steal.py).
//
// Canonical tie-break as in the fixtures: worker_objective gets the worker index as
// its last key; saturated iterates in ascending worker index; each stealable bin in
// ascending task index. Build: oracle/Makefile (-ffp-contract=off).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

namespace {

constexpr int N_LEVELS = 15;       // len(cost_multipliers) (stealing.py:83-85)
constexpr double LATENCY = 0.1;    // stealing.py:37

struct Problem {
  int W;
  const int32_t* nthreads;
  const double* occ;       // WorkerState.occupancy (unchanged during balance)
  const int32_t* nproc;    // len(ws.processing)
  const int64_t* wnbytes;  // ws.nbytes
  double total_occ;        // SchedulerState.total_occupancy
  int64_t total_nthreads;
  int64_t bw;              // scheduler.bandwidth
  int64_t T;
  const int32_t* victim;   // processing_on
  const double* duration;  // get_task_duration(ts)
  const uint8_t* fast;     // prefix in fast_tasks
  const int64_t* dep_ptr;
  const int32_t* dep_idx;  // into the data arrays
  const int64_t* d_nbytes;      // dts.nbytes (raw; get_comm_cost)
  const int64_t* d_get_nbytes;  // dts.get_nbytes() (worker_objective, steal_time_ratio)
  const int64_t* h_ptr;         // who_has of each data task (CSR)
  const int32_t* h_idx;
  // restrictions of the processing tasks (null: none): valid_workers (scheduler.py
  // :3043-3107) as worker indices (CSR); flags bit 0 restricted, bit 1 loose
  const int64_t* r_ptr;
  const int32_t* r_idx;
  const uint8_t* r_flags;
};

bool holds(const Problem& P, int d, int w) {
  for (int64_t k = P.h_ptr[d]; k < P.h_ptr[d + 1]; k++)
    if (P.h_idx[k] == w) return true;
  return false;
}

// steal_time_ratio (stealing.py:241-277) -> level, or -1 for "not stealable"
int steal_level(const Problem& P, int64_t t) {
  if (P.fast[t]) return -1;                         // :252-253
  if (P.dep_ptr[t] == P.dep_ptr[t + 1]) return 0;   // :255-256 no dependencies
  const double compute = P.duration[t];             // :258 get_task_duration
  if (!(compute != 0.0)) return -1;                 // :260-265 long-running
  int64_t nb = 0;                                   // :267 get_nbytes_deps
  for (int64_t k = P.dep_ptr[t]; k < P.dep_ptr[t + 1]; k++) nb += P.d_get_nbytes[P.dep_idx[k]];
  const double transfer = (double)nb / (double)P.bw + LATENCY;  // :268
  const double cm = transfer / compute;                          // :269
  int level = (int)std::nearbyint(std::log2(cm) + 6.0);          // :271 int(round(...)), half-even
  if (level < 1) level = 1;                                      // :273-276
  else if (level >= N_LEVELS) return -1;
  return level;
}

// get_comm_cost (scheduler.py:3006-3022): raw nbytes of dependencies not on w / bandwidth
double comm_cost(const Problem& P, int64_t t, int w) {
  int64_t nb = 0;
  for (int64_t k = P.dep_ptr[t]; k < P.dep_ptr[t + 1]; k++) {
    const int d = P.dep_idx[k];
    if (!holds(P, d, w)) nb += P.d_nbytes[d];
  }
  return (double)nb / (double)P.bw;
}

struct Obj {
  double start;
  int64_t nb;
  int w;
  bool operator<(const Obj& o) const {
    if (start != o.start) return start < o.start;
    if (nb != o.nb) return nb < o.nb;
    return w < o.w;
  }
};

// worker_objective (scheduler.py:3131-3146) + canonical index
Obj objective(const Problem& P, int64_t t, int w) {
  int64_t comm = 0;
  for (int64_t k = P.dep_ptr[t]; k < P.dep_ptr[t + 1]; k++) {
    const int d = P.dep_idx[k];
    if (!holds(P, d, w)) comm += P.d_get_nbytes[d];
  }
  const double stack = P.occ[w] / (double)P.nthreads[w];
  return Obj{stack + (double)comm / (double)P.bw, P.wnbytes[w], w};
}

}  // namespace

extern "C" int orc_steal_balance(
    // workers
    int32_t W, const int32_t* nthreads, const double* occ, const int32_t* nproc, const int64_t* wnbytes,
    const uint8_t* idle_in, const uint8_t* sat_in, double total_occ, int64_t total_nthreads, int64_t bandwidth,
    // processing tasks
    int64_t T, const int32_t* victim, const double* duration, const uint8_t* fast, const int64_t* dep_ptr,
    const int32_t* dep_idx,
    // data (dependencies)
    const int64_t* d_nbytes, const int64_t* d_get_nbytes, const int64_t* h_ptr, const int32_t* h_idx,
    // restrictions (nullable)
    const int64_t* r_ptr, const int32_t* r_idx, const uint8_t* r_flags,
    // the plugin's bins and unconfirmed in-flight accounts (nullable)
    const int8_t* level_in, const double* ifo_in, const int32_t* ift_in,
    // outputs
    int8_t* level_out, int32_t* st_task, int32_t* st_victim, int32_t* st_thief, int32_t* st_level, double* st_cost,
    double* st_occ_victim, double* st_occ_thief, int64_t* n_steals, double* inflight_occ, int32_t* inflight_tasks,
    uint8_t* idle_out, uint8_t* sat_out, uint8_t* checked) {
  const Problem P{W, nthreads, occ, nproc, wnbytes, total_occ, total_nthreads, bandwidth, T, victim, duration,
                  fast, dep_ptr, dep_idx, d_nbytes, d_get_nbytes, h_ptr, h_idx, r_ptr, r_idx, r_flags};
  std::vector<uint8_t> idle(idle_in, idle_in + W), sat(sat_in, sat_in + W);
  std::vector<double> ifo(W, 0.0);
  std::vector<int32_t> ift(W, 0);
  for (int w = 0; w < W; w++) {  // _combined_occupancy / _combined_nprocessing (:505-509)
    if (ifo_in) ifo[w] = ifo_in[w];
    if (ift_in) ift[w] = ift_in[w];
    checked[w] = 0;
  }
  *n_steals = 0;
  // put_key_in_stealable (stealing.py:220-230): bins per (worker, level), ascending task
  std::vector<std::vector<int64_t>> bins((size_t)W * N_LEVELS);
  for (int64_t t = 0; t < T; t++) {
    const int lv = level_in ? (int)level_in[t] : steal_level(P, t);
    level_out[t] = (int8_t)lv;
    if (lv >= 0) bins[(size_t)victim[t] * N_LEVELS + lv].push_back(t);
  }
  auto combined_occ = [&](int w) { return occ[w] + ifo[w]; };          // :505-506
  auto combined_nproc = [&](int w) { return nproc[w] + ift[w]; };      // :508-509
  const double avg = total_occ / (double)total_nthreads;
  auto is_unoccupied = [&](int w, double o, int np) {                  // scheduler.py:2997-3004
    return np < nthreads[w] || o < nthreads[w] * avg / 2;
  };
  auto check_idle_saturated = [&](int w, double o) {                    // scheduler.py:2949-2995
    if (o < 0) o = occ[w];                                              // :2974-2975 (negative -> own occupancy)
    const int p = nproc[w];
    sat[w] = 0;
    if (is_unoccupied(w, o, p)) {
      idle[w] = 1;
    } else {
      idle[w] = 0;
      const int nc = nthreads[w];
      if (p > nc) {
        const double pending = o * (double)(p - nc) / (double)(p * nc);
        if (0.4 < pending && pending > 1.9 * avg) sat[w] = 1;
      }
    }
  };
  // balance (stealing.py:401-503)
  std::vector<uint8_t> thief(W, 0);
  int n_thieves = 0;
  for (int w = 0; w < W; w++)
    if (idle[w]) thief[w] = 1, n_thieves++;
  auto finish = [&]() {
    for (int w = 0; w < W; w++) {
      inflight_occ[w] = ifo[w];
      inflight_tasks[w] = ift[w];
      idle_out[w] = idle[w];
      sat_out[w] = sat[w];
    }
    return 0;
  };
  if (n_thieves == 0 || n_thieves == W) return finish();  // :410-411
  bool live = false;                                        // victims = the live saturated set
  std::vector<int> pv;
  int n_sat = 0;
  for (int w = 0; w < W; w++) n_sat += sat[w];
  if (n_sat) {
    for (int w = 0; w < W; w++)
      if (sat[w]) pv.push_back(w);
  } else {  // topk(10, workers, key=combined occupancy), stable on ties (:415-424)
    std::vector<int> all(W);
    for (int w = 0; w < W; w++) all[w] = w;
    std::stable_sort(all.begin(), all.end(), [&](int a, int b) { return combined_occ(a) > combined_occ(b); });
    for (int i = 0; i < W && i < 10; i++) {
      const int w = all[i];
      if (combined_occ(w) > 0.2 && combined_nproc(w) > nthreads[w] && !thief[w]) pv.push_back(w);
    }
    if (pv.empty()) return finish();
  }
  if (pv.size() < 20) {  // :425-428
    std::stable_sort(pv.begin(), pv.end(), [&](int a, int b) { return combined_occ(a) > combined_occ(b); });
  } else {
    live = true;
  }
  for (int level = 0; level < N_LEVELS; level++) {  // :431
    if (!n_thieves) break;
    std::vector<int> vs;
    if (live) {
      for (int w = 0; w < W; w++)
        if (sat[w]) vs.push_back(w);
    } else {
      vs = pv;
    }
    for (int v : vs) {  // :434
      const std::vector<int64_t>& bin = bins[(size_t)v * N_LEVELS + level];
      if (bin.empty() || !n_thieves) continue;
      for (int64_t t : bin) {  // :439
        if (!n_thieves) break;
        Obj best{0, 0, -1};  // _get_thief (:532-542): min objective over the thieves
        const bool rs = P.r_flags && (P.r_flags[t] & 1);
        if (rs)  // potential_thieves & valid_workers
          for (int64_t k = P.r_ptr[t]; k < P.r_ptr[t + 1]; k++) {
            const int w = P.r_idx[k];
            if (!thief[w]) continue;
            const Obj o = objective(P, t, w);
            if (best.w < 0 || o < best) best = o;
          }
        if (best.w < 0 && (!rs || (P.r_flags[t] & 2)))  // unrestricted, or loose with no valid thief
          for (int w = 0; w < W; w++) {
            if (!thief[w]) continue;
            const Obj o = objective(P, t, w);
            if (best.w < 0 || o < best) best = o;
          }
        if (best.w < 0) continue;  // _get_thief -> None: the task is skipped (:452-454)
        const int th = best.w;
        const double occ_thief = combined_occ(th);
        const double occ_victim = combined_occ(v);
        const double cc_thief = comm_cost(P, t, th);
        const double cc_victim = comm_cost(P, t, v);
        const double compute = duration[t];
        if (occ_thief + cc_thief + compute <= occ_victim - (cc_victim + compute) / 2) {  // :462-465
          // move_task_request (:279-331) -> _add_to_in_flight (:191-199)
          ifo[v] -= compute + cc_victim;
          ifo[th] += compute + cc_thief;
          ift[v] -= 1;
          ift[th] += 1;
          const int64_t k = (*n_steals)++;
          st_task[k] = (int32_t)t;
          st_victim[k] = v;
          st_thief[k] = th;
          st_level[k] = level;
          st_cost[k] = compute + cc_victim;
          st_occ_victim[k] = occ_victim;
          st_occ_thief[k] = occ_thief;
          if (!is_unoccupied(th, combined_occ(th), combined_nproc(th))) {  // :487-493
            thief[th] = 0;
            n_thieves--;
          }
        }
      }
      check_idle_saturated(v, combined_occ(v));  // :498-500
      checked[v] = 1;
    }
  }
  return finish();
}
