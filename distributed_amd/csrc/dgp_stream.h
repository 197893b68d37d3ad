// dgplace stream engine: the completion replay as one dataflow pipeline in a single
// persistent workgroup (gfx950, 16 waves). Included by dgplace.hip after dgp_device.h.
//
// The synthetic executor completes placements in run_id order, so the replay after
// update_graph is ONE ordered stream of completion stimuli r = 0, 1, 2, ... (stimulus r
// completes placement r; it is processed after the stimulus that created placement r).
// Sequential semantics only order stimuli that share a worker: a completion on w, its
// releases (the replicas' holders) and its frontier placements (the candidates of the
// released tasks) read and write only those workers' state, and while the queue is
// non-empty every worker but w is full, so the queue refill touches only w
// (stimulus_queue_slots_maybe_opened :4983 -> decide_worker_rootish_queuing_enabled
// :2195). Everything else is global and handled in order.
//
// Waves (roles):
//   SEQ  sequencer: in stimulus order, turns each finished stimulus' staged placements
//        into placement-log entries (run_id order), resolves the queued tasks its pops
//        took (HeapSet order), appends its records to the record log, frees its slot,
//        counts rounds and takes the per-round snapshots.
//   BLD  builder: per completion, in order, the waiting_on / waiters decrements
//        (_add_to_memory :3298-3314): marks each task with the stimulus that releases
//        it to the frontier (fr_mark) or to "released" (rel_mark).
//   PRE  prefetcher: per stimulus, a 1 KiB descriptor in a global ring: the completing
//        task, its dependencies, the releases and every frontier task with its
//        dependencies' holders and sizes (the candidate set of decide_worker :8571).
//   REG  registrar: in order, copies descriptors into the LDS window (32 slots), folds
//        the prefix EWMA (TaskPrefix.add_duration :977), and registers the stimulus on
//        the workers it touches: mask[w] bit per in-flight slot; the stimulus waits for
//        every earlier in-flight stimulus that shares a worker.
//   WLK  walker: folds the record log in order into SchedulerState's global quantities
//        (_task_prefix_count_global, _network_occ_global -> total_occupancy :1877) and
//        the idle / saturated sets of check_idle_saturated (:2949).
//   EXE  executors (the other waves): pick any ready stimulus and run it on the worker
//        state in LDS; stimuli that read global state run alone, in order.
//
// Included twice by dgplace.hip: namespace st with the 32-slot window and wait-in-place
// claims (DGP_WIN 32, DGP_WAITC 1), namespace st64 with 64 slots and no wait-in-place
// (DGP_ST_NS st64, DGP_WIN 64, DGP_WAITC 0). The engine picks one per graph (dgp_set_window).

#include "dgp_svcmsg.h"

#ifndef DGP_ST_NS
#define DGP_ST_NS st
#endif

#ifndef DGP_STREAM_SHARED_DEFINED
#define DGP_STREAM_SHARED_DEFINED
#define DGP_ST_PRIMARY 1  // the first inclusion also defines the window-independent kernels
namespace dgp {
// the stream kernel's static LDS block (SLds), one allocation for both window builds in the
// module-wide LDS struct, sized for the 64-slot one (each namespace checks its SLds fits)
constexpr size_t ST_LDS_BYTES = 22608;
__shared__ __attribute__((aligned(16))) char st_lds_raw[ST_LDS_BYTES];
// the per-worker LDS carve (dynamic LDS, sized at launch)
extern __shared__ __attribute__((aligned(16))) char st_smem[];
}  // namespace dgp
#else
#undef DGP_ST_PRIMARY
#define DGP_ST_PRIMARY 0
#endif

namespace dgp {
namespace DGP_ST_NS {

// the engine description every stream role reads: constant memory (scalar loads, never
// re-fetched across the roles' fences); set by the host before each launch
__constant__ Dev c_dev;

#ifndef DGP_PHASE_PROBES
#define DGP_PHASE_PROBES 0  // per-phase s_memtime probes in the executors (diagnostics)
#endif
#ifndef DGP_EXE_PRIO
#define DGP_EXE_PRIO 1  // 0: fixed priority 2; 1 / 2: executors issue at priority 3 while running a stimulus, 1 / 0 while polling
#endif
#ifndef DGP_EXE_SLEEP
#define DGP_EXE_SLEEP 1  // s_sleep units (64 clocks) between an idle executor's polls
#endif
#ifndef DGP_EXE_PF
#define DGP_EXE_PF 1  // an idle executor loads the descriptor of the oldest waiting stimulus ahead of its claim
#endif
#ifndef DGP_PROF_GLOBAL
#define DGP_PROF_GLOBAL 0  // diagnostics (with DGP_PROF): prof[9] / [22] take cycles of global stimuli / wide fan-ins
#endif
#ifndef DGP_REG_PROBES
#define DGP_REG_PROBES 0  // registrar sub-phase s_memtime probes (diagnostics)
#endif
#ifndef DGP_BULK_RESTR
#define DGP_BULK_RESTR 1  // global frontier: restricted single-worker tasks on distinct workers placed lane-parallel
#endif
#ifndef DGP_RUN_PAR
#define DGP_RUN_PAR 1  // single-worker runs of one prefix: every member's record at once (lane = member)
#endif
#ifndef DGP_RB
#define DGP_RB 8  // registrar batch (stimuli registered per poll, one lane each)
#endif
#ifndef DGP_SCTA
#define DGP_SCTA 1024
#endif
constexpr int SCTA = DGP_SCTA;   // 1024: 16 waves = 5 roles + 11 executors (128 VGPRs per wave; 768/7 executors: C2 1.18 s, 1024: 1.14 s)
#ifndef DGP_WIN
#define DGP_WIN 32
#endif
constexpr int WIN = DGP_WIN;     // in-flight stimulus slots (LDS window; masks are u64: <= 64)
using SMask = unsigned long long;  // a set of window slots
static_assert(WIN >= 32 && WIN <= 64, "DGP_WIN must be in [32, 64]");
#ifndef DGP_WAITC
// 1: a stimulus is claimed once its completing worker and release holders are free and waits
// in place for its frontier candidates (predc) just before its frontier; 0: claimed only
// once every touched worker is free
#define DGP_WAITC 1
#endif
constexpr bool WAITC = DGP_WAITC != 0;
// a stimulus that would wait in place is claimed only within this many stimuli of the oldest
// (stimuli in flight span up to RS; 4 / 8 / 16 / 20 measured slower, profiles/r04knob)
constexpr int WAITC_AHEAD = 32;
static_assert(!WAITC || WIN == 32, "DGP_WAITC keeps the candidate-only registrations in the masks' high half");
// the mask bits of slot s: its registration (low half) and, with WAITC, the candidate-only
// flag of this worker for s (high half)
__host__ __device__ constexpr unsigned long long slot_bits(int s) {
  return WAITC ? ((1ull << s) | (1ull << (s + 32))) : (1ull << s);
}
#ifndef DGP_RS
#define DGP_RS 128
#endif
// retire ring: stimuli registered but not yet sequenced. A slot is held only while its
// stimulus is registered and running; a finished stimulus leaves its counts here (and its
// outputs in the staging rows of r & (RS - 1)) until the sequencer retires it in order.
constexpr int RS = DGP_RS;
constexpr int NE = 64;           // 16-byte descriptor entries per stimulus (one per lane)
#ifndef DGP_DR
// 512 rows x (64 x 16 B descriptor + 32 x 4 B touch list) = 576 KB stays in L2: PMC read
// traffic 1.31 -> 0.18 GB per C2 replay, same time
#define DGP_DR 512
#endif
constexpr int DR = DGP_DR;       // descriptor ring (global) — how far PRE may run ahead
constexpr int PLC = 64;          // staged placements / records per stimulus
constexpr int KT_MAX = 24;       // dependencies of the completing task in local mode
constexpr int KX_MAX = 8;        // dependencies of a frontier task in local mode
constexpr int RC_MAX = 8;        // decide_worker candidates of a restricted frontier task in local mode
constexpr int PD = 8;            // entries of one worker's prefix dict (PMAX): the descriptor's 8 durations serve P <= PD
constexpr int PX = 32;           // task prefixes the stream engine takes (P > PD: durations in rows of D.dring)
constexpr int TMAX = 32;         // distinct workers a local stimulus may touch (more: global)
constexpr int NLW = 12;          // needs_what words per worker in LDS: 11 entries + control
constexpr int NXW = 52;          // overflow entries per worker (global) before scan mode
constexpr int PG = 64;           // walker's global prefix dict
constexpr int BIG = 1 << 24;     // registration guard of a slot's predecessor count
constexpr int T_CAND = 0x8000;   // touch-list entry flag: the worker is a frontier candidate (ids < 32768)
constexpr int T_W = 0x7fff;
constexpr uint32_t NL_OVF = 0xffffffffu;
static_assert(NLW == SNLW && NXW == SNXW && NL_OVF == SNL_OVF, "dgp_device.h's one-lane needs_what ops use this layout");
constexpr int N_ROLE = 5;        // waves 0..4 are SEQ, BLD, PRE, REG, WLK; the rest execute
constexpr int E_HDR = 7;         // header entries: 0 ids, 1 sizes/counts, 2 duration, 3..6 durations
// rows are selected with r & (DR - 1); PRE runs at most DR ahead and at least one window
static_assert((DR & (DR - 1)) == 0 && DR >= 64 && DR >= WIN, "DGP_DR must be a power of two >= 64");
static_assert((RS & (RS - 1)) == 0 && RS >= WIN && RS <= DR, "DGP_RS must be a power of two in [WIN, DR]");

// F_SIMPLE (PRE): touches only its completing worker, empty frontier, at most one dependency
// (held by that worker, or by another one and not released) and one release: it can be part
// of a single-worker run (exe_run).
// F_RUNM (REG): F_SIMPLE and so is the stimulus just before it, on the same worker: a run
// continues through it, so only the run-capable executor takes it
enum : uint32_t { F_GLOBAL = 1, F_SELFREL = 2, F_EXACT = 4, F_TOUCHALL = 8, F_BADTOUCH = 16, F_SIMPLE = 32, F_RUNM = 64 };
// K_COMPLETE_LR: the completion of a long-running task (its prefix count left the worker's and
// the global dict at add_to_long_running :747-757; remove_from_processing :764-766)
enum : int { K_COMPLETE = 1, K_PLACE = 2, K_COMPLETE_LR = 3 };
enum : int { SERR_NONE = 0, SERR_PREFIX = 11, SERR_WATCHDOG = 12, SERR_QUEUE = 13, SERR_NEEDS = 14,
             SERR_REC = 15, SERR_CAND = 16, SERR_STAGE = 17, SERR_RANGE = 18, SERR_INV = 19 };

#if DGP_ST_PRIMARY  // Dev points at these (dgp_device.h): one type for both builds
// persistent stream position (global, survives launches)
struct Pos {
  long long seq, bld, pre, reg;  // stimuli sequenced / built / prefetched / registered
  long long rec_len, walk;       // record log length / records folded
  long long runid_upto;          // placement-log entries whose run_id / holder are set
  long long round_end;           // end of the current round (stimulus index), -1 before the first launch
  long long round_start_saved;   // start of the current round
  long long prev_placed;         // log length at the last snapshot
};

// one record of the record log (one check_idle_saturated sub-step)
struct SRec {
  int32_t w;
  int16_t p;
  int8_t kind;
  int8_t pad;
  int32_t nproc;
  int32_t task;
  int64_t dnet;
  double occ;
  double dur;  // completion: the observed duration (stop - start) for the prefix EWMA
};
#else
using st::Pos;
using st::SRec;
#endif

// LDS control block
struct SCtl {
  int stop, error, err_task;
  int inv_ok;          // queue non-empty => every worker full (only globals change it)
  int q_anon;          // queued tasks share one prefix and have no dependencies
  int q_prefix;
  int capmax;          // max slot cap over workers
  int global_pending;  // a registered global stimulus has not finished
  int busy_exe;        // executors between claim and retirement
  SMask ready;         // slots whose stimulus may run
  SMask freem;         // slots not holding a registered stimulus (REG allocates, executors free)
  long long seq_pos, log_len, rec_len, walk_pos, bld_pos, pre_pos, reg_pos, reg_limit;
  long long qhead, qlen, n_tasks;
  long long stim_end;  // service mode: stimuli [seq_pos, stim_end) run in this launch
  unsigned long long t_role[8];  // resident mode: when each role last finished a batch (100 MHz clock)
  long long req_n, req_off, req_pl0;  // resident service: the request's messages, consumed, first placement
  unsigned long long req_seen;        // resident service: the last request taken
  long long round_end, rounds_left, prev_placed;
  long long rounds_nonempty, snap_idx;
  int snaps;
  // walker state (SchedulerState globals as of walk_pos)
  int g_plen;
  int g_pfx[PG];
  long long g_pcnt[PG];
  double g_netocc;
  double wdur[PX];  // prefix EWMA as of walk_pos (raw duration_average)
  long long n_idle, n_sat;
  unsigned long long prof[32];
};

// ------------------------------------------------------------------ small helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ unsigned rlu(unsigned v, int l) { return (unsigned)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ int64_t mk64(unsigned lo, unsigned hi) { return (int64_t)(((uint64_t)hi << 32) | lo); }
__device__ __forceinline__ double mkd(unsigned lo, unsigned hi) {
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ unsigned lo32(int64_t v) { return (unsigned)(uint64_t)v; }
__device__ __forceinline__ unsigned hi32(int64_t v) { return (unsigned)((uint64_t)v >> 32); }
__device__ __forceinline__ unsigned dlo(double v) { return lo32(__double_as_longlong(v)); }
__device__ __forceinline__ unsigned dhi(double v) { return hi32(__double_as_longlong(v)); }
__device__ __forceinline__ int64_t shfl64(int64_t v, int l) { return __shfl(v, l); }
__device__ __forceinline__ int64_t wsum64(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int wsum(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int wmax(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ unsigned long long ballot(bool b) { return __ballot(b); }
// Profiling clock and counters (dgp_stats wave_phase* / stall*): only in DGP_PROF builds.
// s_memtime is a scalar memory read that waits on the LDS counter (lgkmcnt), so every probe
// would drain the wave's outstanding LDS operations on the hot paths.
#ifndef DGP_PROF
#define DGP_PROF 0
#endif
__device__ __forceinline__ unsigned long long mclk() { return DGP_PROF ? __builtin_amdgcn_s_memtime() : 0ull; }
// DGP_TRACE builds: lifecycle timestamps of sampled stimuli (tools/trace_analyze.py):
// 0 registered, 1 ready, 2 claimed, 3 early release, 4 non-w release, 5 done, 6 retired,
// 7 predecessor count | touched workers << 16 | executor wave << 24.
// DGP_TRACE=3: those, plus the executor's phases and who made the stimulus ready
// (tools/link_profile.py): 8 precheck, 9 state loaded, 10 completion needs, 11 before the
// wait, 12 after the wait, 13 first frontier keys, 14 argmin + early release, 15 first commit,
// 16 frontier done, 17 refill done, 18 w released, 19 the stimulus whose release made it
// ready, 20 candidates final (predc 0), 21 the stimulus whose release did that,
// 22 nf | kt << 8 | nrel << 16 | nt << 24, 23 predc at the claim. One row is DGP_TSTR words.
#ifndef DGP_TRACE
#define DGP_TRACE 0
#endif
constexpr int TSTR = 32;
constexpr bool TRL = DGP_TRACE == 1 || DGP_TRACE == 3;  // lifecycle events
constexpr bool TR3 = DGP_TRACE == 3;                     // executor phases
__device__ __forceinline__ void trace_at(const Dev& D, long long r, int k, unsigned long long v) {
  if (DGP_TRACE && D.trace && r >= D.trace_lo && r < D.trace_lo + D.trace_n) D.trace[(r - D.trace_lo) * TSTR + k] = v;
}
#define TR(r, k) trace_at(D, (r), (k), __builtin_amdgcn_s_memtime())
#define PROF(stmt) \
  do {             \
    if (DGP_PROF) { stmt; } \
  } while (0)
__device__ __forceinline__ void wbar() { __builtin_amdgcn_wave_barrier(); }
__device__ __forceinline__ void lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

template <class T>
__device__ __forceinline__ T vload(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <class T>
__device__ __forceinline__ void vstore(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ------------------------------------------------------------ worker state access
// LW: state in LDS (dynamic carve, ds_* instructions), else in the global gw_* arrays
template <bool LW>
struct AS {
  template <class T>
  using P = T*;
};
template <>
struct AS<true> {
  template <class T>
  using P = __attribute__((address_space(3))) T*;
};

template <bool LW>
struct WPtr {
  template <class T>
  using P = typename AS<LW>::template P<T>;
  P<int32_t> nproc;
  P<uint16_t> nthreads;
  P<uint16_t> cap;
  P<uint32_t> plen;    // prefix dict insertion order (WDict::ord)
  P<uint32_t> pcnt;    // [W][PD] prefix dict counts by prefix id (WDict::c, c1)
  P<int64_t> netocc;
  P<int64_t> nbytes;
  P<SMask> mask;       // in-flight slots touching the worker
  P<uint32_t> needs;   // [W][NLW]: (d << 8 | count), slot NLW-1 = control (count << 8 | 1 when
                       // overflow entries are in use; NL_OVF: scan mode)
  P<uint8_t> wflags;   // walker's idle / saturated bits
};


__device__ __forceinline__ size_t al16(size_t b) { return (b + 15) & ~(size_t)15; }
__host__ __device__ constexpr size_t lds_worker_bytes(int W) {
  return ((size_t)W * 4 + 15) / 16 * 16 * 2 /* nproc plen */ + ((size_t)W * 2 + 15) / 16 * 16 * 2 +
         ((size_t)W * PD * 4 + 15) / 16 * 16 + ((size_t)W * 8 + 15) / 16 * 16 * 2 +
         ((size_t)W * 8 + 15) / 16 * 16 + ((size_t)W * NLW * 4 + 15) / 16 * 16 + ((size_t)W + 15) / 16 * 16;
}

template <bool LW>
__device__ __forceinline__ WPtr<LW> wptr(const Dev& D) {
  WPtr<LW> p;
  using W_ = WPtr<LW>;
  if constexpr (LW) {
    const size_t W = D.W;
    auto b = (__attribute__((address_space(3))) char*)st_smem;
    p.nproc = (typename W_::template P<int32_t>)b;     b += al16(W * 4);
    p.nthreads = (typename W_::template P<uint16_t>)b; b += al16(W * 2);
    p.cap = (typename W_::template P<uint16_t>)b;      b += al16(W * 2);
    p.plen = (typename W_::template P<uint32_t>)b;     b += al16(W * 4);
    p.pcnt = (typename W_::template P<uint32_t>)b;     b += al16(W * PD * 4);
    p.netocc = (typename W_::template P<int64_t>)b;    b += al16(W * 8);
    p.nbytes = (typename W_::template P<int64_t>)b;    b += al16(W * 8);
    p.mask = (typename W_::template P<SMask>)b;        b += al16(W * 8);
    p.needs = (typename W_::template P<uint32_t>)b;    b += al16(W * NLW * 4);
    p.wflags = (typename W_::template P<uint8_t>)b;
  } else {
    p.nproc = D.gw_nproc;
    p.nthreads = D.gw_nthreads;
    p.cap = D.gw_cap;
    p.plen = D.gw_plen;
    p.pcnt = D.gw_pcnt;
    p.netocc = D.gw_netocc;
    p.nbytes = D.gw_nbytes;
    p.mask = D.gw_mask;
    p.needs = D.gw_needs;
    p.wflags = D.gw_wflags;
  }
  return p;
}

template <class T, class U>
__device__ __forceinline__ T ascast(U p) {
  return (T)p;
}
struct alignas(16) Q4 {  // plain 16-byte word (uint4 cannot bind an LDS lvalue)
  uint32_t x, y, z, w;
};
template <class PQ>
__device__ __forceinline__ uint4 ld4(PQ q) {
  return make_uint4(q->x, q->y, q->z, q->w);
}
template <class PQ>
__device__ __forceinline__ void st4(PQ q, const uint4& u) {
  q->x = u.x;
  q->y = u.y;
  q->z = u.z;
  q->w = u.w;
}

// what the sequencer needs of a finished stimulus
struct RMeta {
  int32_t npl;                 // placements staged (a global stimulus: written to the log directly)
  uint8_t nrec, npops, direct, pad;
};

// LDS of the stream kernel besides the worker carve
struct SLds {
  double dur[SCTA / 64][PX];  // each executor wave: its stimulus' resolved prefix durations
  uint16_t touch[WIN][NE];    // distinct workers each in-flight stimulus touches (| T_CAND)
  int32_t ntouch[WIN];
  uint32_t flags[WIN];
  int32_t pred[WIN];
  int32_t predc[WIN];         // WAITC: frontier candidates an earlier in-flight stimulus still holds
  long long sid[WIN];         // stimulus registered in each slot
  RMeta rmeta[RS];            // retire ring: counts of finished stimulus r at r & (RS - 1)
  long long rdone[RS];        // ... and r + 1 once they are final
  uint16_t pre_scr[64][TMAX]; // prefetcher scratch: each lane's distinct-worker list
  int32_t bld_jobs[256];      // builder: wide rows deferred to the whole wave (kind << 28 | task)
  int32_t bld_njobs;
  SCtl c;
};

static_assert(sizeof(SLds) <= ST_LDS_BYTES, "ST_LDS_BYTES must hold the 64-slot window's SLds");
// the engine's LDS window + control block (namespace scope: the roles' out-of-line entry
// functions address it directly, keeping ds_* addressing)
__device__ __forceinline__ SLds& st_L() { return *reinterpret_cast<SLds*>(st_lds_raw); }

// ---------------------------------------------------------- the per-worker prefix dict
// WorkerState.task_prefix_count is an insertion-ordered {prefix: count} with delete on
// zero (:733-784). Held as up to PD slots in insertion order, slot i = prefix id << 24 |
// count (ids < 256, counts < 2^24) in 8 words (c: slots 0..3, c1: slots 4..7); ord >> 24
// is the number of entries. A prefix is present iff it has a slot, so this is the dict.
struct WDict {
  uint4 c, c1;   // the slots
  uint32_t ord;  // entries << 24
};
__device__ __forceinline__ uint32_t wd_n(uint32_t ord) { return ord >> 24; }
__device__ __forceinline__ uint32_t wd_slot(const WDict& d, int i) {
  switch (i & 7) {
    case 0: return d.c.x;
    case 1: return d.c.y;
    case 2: return d.c.z;
    case 3: return d.c.w;
    case 4: return d.c1.x;
    case 5: return d.c1.y;
    case 6: return d.c1.z;
    default: return d.c1.w;
  }
}
__device__ __forceinline__ void wd_put(WDict& d, int i, uint32_t v) {
  switch (i & 7) {
    case 0: d.c.x = v; break;
    case 1: d.c.y = v; break;
    case 2: d.c.z = v; break;
    case 3: d.c.w = v; break;
    case 4: d.c1.x = v; break;
    case 5: d.c1.y = v; break;
    case 6: d.c1.z = v; break;
    default: d.c1.w = v; break;
  }
}
__device__ __forceinline__ int wd_find(const WDict& d, int p) {  // slot of prefix p, -1: absent
  const uint32_t n = wd_n(d.ord);
  int k = -1;
#pragma unroll
  for (int i = 0; i < PD; i++)
    if ((uint32_t)i < n && (wd_slot(d, i) >> 24) == (uint32_t)p) k = i;
  return k;
}
__device__ __forceinline__ uint32_t wd_cnt(const WDict& d, int p) {
  const int k = wd_find(d, p);
  return k < 0 ? 0u : (wd_slot(d, k) & 0xffffffu);
}
// count of prefix p := v > 0 (its slot, or a new one appended)
__device__ __forceinline__ void wd_set(WDict& d, int p, uint32_t v) {
  int k = wd_find(d, p);
  if (k < 0) {
    k = (int)wd_n(d.ord);
    d.ord += 1u << 24;
  }
  wd_put(d, k, ((uint32_t)p << 24) | (v & 0xffffffu));
}

// add_to_processing (+1) / remove_from_processing (-1) of one task of prefix p
__device__ __forceinline__ bool dict_add(WDict& d, int p, int delta) {
  const int k = wd_find(d, p);
  const uint32_t n = wd_n(d.ord);
  if (delta > 0) {
    if (k >= 0) {
      const uint32_t v = wd_slot(d, k);
      if ((v & 0xffffffu) == 0xffffffu) return false;
      wd_put(d, k, v + 1u);
      return true;
    }
    if (n >= (uint32_t)PD || p < 0 || p > 255) return false;
    wd_put(d, (int)n, ((uint32_t)p << 24) | 1u);  // new key: appended
    d.ord += 1u << 24;
    return true;
  }
  if (k < 0) return true;
  const uint32_t v = wd_slot(d, k);
  if ((v & 0xffffffu) > 1u) {
    wd_put(d, k, v - 1u);
    return true;
  }
  // count reached zero: the key leaves, later keys move up
#pragma unroll
  for (int i = 0; i < PD - 1; i++)
    if (i >= k) wd_put(d, i, wd_slot(d, i + 1));
  wd_put(d, PD - 1, 0u);
  d.ord -= 1u << 24;
  return true;
}

// add_to_processing (+1) / remove_from_processing (-1) of prefix p on lane j's dict only
// (uniform j): lane j's slots read once, the insertion-ordered update (dict_add's) on
// scalar registers, the slots written back to lane j (one select each)
__device__ __forceinline__ bool dict_add_lane(WDict& d, int j, int p, int delta) {
  uint32_t sl[PD] = {rlu(d.c.x, j), rlu(d.c.y, j), rlu(d.c.z, j), rlu(d.c.w, j),
                     rlu(d.c1.x, j), rlu(d.c1.y, j), rlu(d.c1.z, j), rlu(d.c1.w, j)};
  uint32_t ord = rlu(d.ord, j);
  const uint32_t n = ord >> 24;
  int k = -1;
#pragma unroll
  for (int i = 0; i < PD; i++)
    if ((uint32_t)i < n && (sl[i] >> 24) == (uint32_t)p) k = i;
  bool ok = true;
  if (delta > 0) {
    if (k >= 0) {
#pragma unroll
      for (int i = 0; i < PD; i++)
        if (i == k) {
          if ((sl[i] & 0xffffffu) == 0xffffffu) ok = false;
          else sl[i] += 1u;
        }
    } else if (n >= (uint32_t)PD || p < 0 || p > 255) {
      ok = false;
    } else {
#pragma unroll
      for (int i = 0; i < PD; i++)
        if (i == (int)n) sl[i] = ((uint32_t)p << 24) | 1u;  // new key: appended
      ord += 1u << 24;
    }
  } else if (k >= 0) {
    uint32_t ck = 0;
#pragma unroll
    for (int i = 0; i < PD; i++)
      if (i == k) ck = sl[i] & 0xffffffu;
    if (ck > 1u) {
#pragma unroll
      for (int i = 0; i < PD; i++)
        if (i == k) sl[i] -= 1u;
    } else {  // count reached zero: the key leaves, later keys move up
#pragma unroll
      for (int i = 0; i < PD - 1; i++)
        if (i >= k) sl[i] = sl[i + 1];
      sl[PD - 1] = 0u;
      ord -= 1u << 24;
    }
  }
  const bool lj = lane_id() == j;
  d.c.x = lj ? sl[0] : d.c.x;
  d.c.y = lj ? sl[1] : d.c.y;
  d.c.z = lj ? sl[2] : d.c.z;
  d.c.w = lj ? sl[3] : d.c.w;
  d.c1.x = lj ? sl[4] : d.c1.x;
  d.c1.y = lj ? sl[5] : d.c1.y;
  d.c1.z = lj ? sl[6] : d.c1.z;
  d.c1.w = lj ? sl[7] : d.c1.w;
  d.ord = lj ? ord : d.ord;
  return ok;
}

// prefix durations: a table of PX doubles in LDS (a descriptor's entries 3..6 or a D.dring
// row, or the walker's wdur), read by prefix id
using DTab = const __attribute__((address_space(3))) double*;

__device__ __forceinline__ double resolve_dur(const Dev& D, double d, int p) {  // _calc_occupancy :1892-1899
  return d < 0 ? (D.pmaxexec[p] > 0 ? 2 * D.pmaxexec[p] : D.unknown_duration) : d;
}

// _calc_occupancy (:1884-1903): prefix terms in dict order, then network occupancy.
// Durations resolve as there (EWMA, else 2 max_exec_time, else unknown-task-duration;
// idempotent on resolved).
__device__ __forceinline__ double occ_dict(const WDict& d, int64_t netocc, DTab dt, const Dev& D) {
  const uint32_t n = wd_n(d.ord);
  double res = 0.0;
#pragma unroll
  for (int i = 0; i < PD; i++) {
    if (!ballot((uint32_t)i < n)) break;
    const uint32_t v = wd_slot(d, i);
    const int p = (int)(v >> 24) & (PX - 1);
    const double dv = dt[p];
    const double term = resolve_dur(D, dv, p) * (double)(v & 0xffffffu);
    if ((uint32_t)i < n) res += term;
  }
  return res + (double)netocc / (double)D.bandwidth;
}

// The executors' form of occ_dict: the network term netocc / bandwidth is carried per
// lane (recomputed only when netocc changes). The same fp64 operations in the same order:
// bit-identical to occ_dict.
__device__ __forceinline__ double occ_dict_r(const WDict& d, double net_bw, DTab dt, const Dev& D) {
  const uint32_t n = wd_n(d.ord);
  double res = 0.0;
  // the first two entries' duration loads issued together (most workers hold at most two
  // prefixes), then the rest one at a time; the same fp64 operations in dict order
  {
    const uint32_t v0 = d.c.x, v1 = d.c.y;
    const double dv0 = dt[(v0 >> 24) & (PX - 1)], dv1 = dt[(v1 >> 24) & (PX - 1)];
    const double t0 = (dv0 < 0 ? D.unknown_duration : dv0) * (double)(v0 & 0xffffffu);
    const double t1 = (dv1 < 0 ? D.unknown_duration : dv1) * (double)(v1 & 0xffffffu);
    if (n > 0u) res += t0;
    if (n > 1u) res += t1;
  }
#pragma unroll
  for (int i = 2; i < PD; i++) {
    if (!ballot((uint32_t)i < n)) break;
    const uint32_t v = wd_slot(d, i);
    const double dv = dt[(v >> 24) & (PX - 1)];
    const double term = (dv < 0 ? D.unknown_duration : dv) * (double)(v & 0xffffffu);
    if ((uint32_t)i < n) res += term;
  }
  return res + net_bw;
}
__device__ __forceinline__ double net_bw_of(int64_t netocc, const Dev& D) {
  return (double)netocc / (double)D.bandwidth;
}

template <bool LW>
__device__ __forceinline__ WDict dict_load(const WPtr<LW>& P, int c) {
  using U4 = typename WPtr<LW>::template P<const Q4>;
  WDict d;
  d.c = ld4(ascast<U4>(P.pcnt + (size_t)c * PD));
  d.c1 = ld4(ascast<U4>(P.pcnt + (size_t)c * PD + 4));
  d.ord = P.plen[c];
  return d;
}

// occupancy of worker c (per lane; any lanes)
template <bool LW>
__device__ __forceinline__ double occ_of(const WPtr<LW>& P, const Dev& D, int c, DTab dt) {
  return occ_dict(dict_load<LW>(P, c), P.netocc[c], dt, D);
}


__device__ __attribute__((always_inline)) void serr(SCtl& S, int code, int task) {
  if (atomicCAS(&S.error, 0, code) == 0) S.err_task = task;
  vstore(&S.stop, 1);
}


// The watchdog runs on s_memrealtime, the constant 100 MHz counter (s_memtime is the
// shader clock: its rate follows the power state, and one read was seen to go backwards
// during a C5 replay). 16 s without progress stops the engine with SERR_WATCHDOG.
constexpr unsigned long long WATCHDOG = 1600000000ull;  // s_memrealtime ticks (100 MHz): 16 s
__device__ __forceinline__ unsigned long long rclk() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ bool stalled_for(unsigned long long since, unsigned long long now) {
  return now - since > WATCHDOG;
}

__device__ __forceinline__ int64_t nbv(const Dev& D, int64_t v) { return v >= 0 ? v : D.default_data_size; }
// w in valid_workers(ts) (:3043-3107) as resolved on the host: task x's restriction row (ascending)
__device__ __forceinline__ bool restr_has(const Dev& D, int x, int w) {
  const RRow rr = restr_row(D, x);
  int64_t lo = rr.r0, hi = rr.r1;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rr.idx[mid] < w) lo = mid + 1;
    else hi = mid;
  }
  return lo < rr.r1 && rr.idx[lo] == w;
}

// ============================================================ walker (records -> flags)
// SchedulerState globals folded in record order, held in registers: the insertion-ordered
// _task_prefix_count_global with entry i in lane i, lane p holding the raw duration_average
// of prefix p; the rest uniform over lanes.
struct WState {
  int n;             // _task_prefix_count_global entries (uniform)
  int pf;            // lane i < n: prefix id of entry i
  long long cnt;     // lane i < n: its count
  double netocc;     // _network_occ_global (holds integers < 2^53: exact in any order)
  double wd;         // lane p: TaskPrefix.duration_average
  long long n_idle, n_sat;
};
static_assert(PG == 64 && PX <= 64, "one lane per global dict entry / per prefix");

__device__ __forceinline__ int64_t rl_i64(int64_t v, int l) { return mk64(rlu(lo32(v), l), rlu(hi32(v), l)); }
__device__ __forceinline__ double rl_f64(double v, int l) { return mkd(rlu(dlo(v), l), rlu(dhi(v), l)); }

__device__ __forceinline__ void ws_load(const SCtl& S, WState& g) {
  const int lane = lane_id();
  g.n = S.g_plen;
  g.pf = S.g_pfx[lane];
  g.cnt = S.g_pcnt[lane];
  g.netocc = S.g_netocc;
  g.wd = S.wdur[lane & (PX - 1)];
  g.n_idle = S.n_idle;
  g.n_sat = S.n_sat;
}
__device__ __forceinline__ void ws_store(SCtl& S, const WState& g) {
  const int lane = lane_id();
  if (lane == 0) {
    S.g_plen = g.n;
    S.g_netocc = g.netocc;
    S.n_idle = g.n_idle;
    S.n_sat = g.n_sat;
  }
  S.g_pfx[lane] = g.pf;
  S.g_pcnt[lane] = g.cnt;
  if (lane < PX) S.wdur[lane] = g.wd;
}
__device__ __forceinline__ bool gdict_add(WState& g, int p, int delta) {
  const int lane = lane_id();
  const unsigned long long m = ballot(lane < g.n && g.pf == p);
  if (delta > 0) {
    if (m) {
      if (lane == __builtin_ctzll(m)) g.cnt++;
      return true;
    }
    if (g.n >= PG) return false;
    if (lane == g.n) {
      g.pf = p;
      g.cnt = 1;
    }
    g.n++;
    return true;
  }
  if (!m) return true;
  const int at = __builtin_ctzll(m);
  const long long v = rl_i64(g.cnt, at) - 1;
  if (v > 0) {
    if (lane == at) g.cnt = v;
    return true;
  }
  // the entry leaves: later entries move up one lane
  const int pn = __shfl_down(g.pf, 1);
  const long long cn = __shfl_down(g.cnt, 1);
  if (lane >= at) {
    g.pf = pn;
    g.cnt = cn;
  }
  g.n--;
  return true;
}
// lane p: prefix p's duration as _calc_occupancy resolves it
__device__ __forceinline__ double ws_lane_dur(const Dev& D, const WState& g) {
  const int lane = lane_id();
  return lane < D.P ? resolve_dur(D, g.wd, lane) : -1.0;
}
// SchedulerState.total_occupancy :1877 (prefix dict order)
__device__ __forceinline__ double ws_total_occ(const Dev& D, const WState& g) {
  const double dv = __shfl(ws_lane_dur(D, g), g.pf & 63);  // entry lane: its prefix's duration
  const double term = dv * (double)g.cnt;
  double res = 0.0;
  for (int i = 0; i < g.n; i++) res += rl_f64(term, i);
  return res + g.netocc / (double)D.bandwidth;
}

// one record: the global-count update of its sub-step, then check_idle_saturated's idle /
// saturated part for its worker (:2949-2991, is_unoccupied :2997). All lanes, uniform.
template <bool LW>
__device__ __forceinline__ void ws_fold(const Dev& D, const WPtr<LW>& P, SCtl& S, WState& g, int kind, int w, int p,
                                        long long dnet, double occ, int nproc, double dobs) {
  const int lane = lane_id();
  if (kind != K_PLACE) {
    // no compute interval in the message (NaN): no EWMA step (TaskGroup.add_duration :1114)
    if (lane == p && dobs == dobs) g.wd = g.wd < 0 ? dobs : 0.5 * dobs + 0.5 * g.wd;
    if (kind == K_COMPLETE) gdict_add(g, p, -1);
  } else if (!gdict_add(g, p, +1)) {
    serr(S, SERR_PREFIX, -1);
  }
  g.netocc += (double)dnet;
  const long long nt = P.nthreads[w];
  const long long pp = nproc;
  bool idle, sat = false;
  double avg = -1.0;
  const bool paused = (P.wflags[w] & WF_PAUSED) != 0;
  if (paused) {
    idle = false;  // not running: idle.pop, saturated.discard (:2975-2977)
  } else if (pp < nt) {
    idle = true;
  } else {
    avg = ws_total_occ(D, g) / (double)D.total_nthreads;
    idle = occ < (double)nt * avg / 2;
  }
  if (!idle && pp > nt && !paused) {
    const double pending = occ * (double)(pp - nt) / (double)(pp * nt);
    if (0.4 < pending) {
      if (avg < 0) avg = ws_total_occ(D, g) / (double)D.total_nthreads;
      sat = pending > 1.9 * avg;
    }
  }
  const uint8_t fo = P.wflags[w];
  const uint8_t fn = (fo & WF_PAUSED) | (idle ? WF_IDLE : 0) | (sat ? WF_SAT : 0);
  if (fo != fn) {
    g.n_idle += (idle ? 1 : 0) - ((fo & WF_IDLE) ? 1 : 0);
    g.n_sat += (sat ? 1 : 0) - ((fo & WF_SAT) ? 1 : 0);
    if (lane == 0) P.wflags[w] = fn;
  }
}

__device__ __forceinline__ long long wscan_incl(long long v) {
  const int lane = lane_id();
  for (int o = 1; o < 64; o <<= 1) {
    const long long u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}

// fold a batch of m records (lane i holds record i). Fast path, all records at once:
// no prefix EWMA changes value and no prefix enters / leaves the global dict in the
// batch, so every record's total_occupancy is a prefix sum over the lanes (integer
// counts, integer-valued network bytes: exact in any order). Otherwise one by one.
template <bool LW>
__device__ __attribute__((always_inline)) void ws_fold_batch(const Dev& D, const WPtr<LW>& P, SCtl& S, WState& g,
                                                             const SRec& rc, int m) {
  const int lane = lane_id();
  const bool in = lane < m;
  const int kind = rc.kind, w = rc.w, p = rc.p, np = rc.nproc;
  // (a) durations unchanged: every completion's EWMA result equals the current value
  const double cur = __shfl(g.wd, p & 63);
  const double nw = cur < 0 ? rc.dur : 0.5 * rc.dur + 0.5 * cur;
  bool bad = in && kind != K_PLACE && rc.dur == rc.dur && __double_as_longlong(nw) != __double_as_longlong(cur);
  // (b) prefix counts stay >= 1 and every record's prefix is in the dict; meanwhile each
  // record lane's prefix terms of total_occupancy in dict order (used when not bad)
  bool found = !in;
  long long tot_mine = 0;  // entry lane k: the batch's count change of entry k
  const double dvl = __shfl(ws_lane_dur(D, g), g.pf & 63);  // entry lane k: its prefix's duration
  double tocc = 0.0;
  for (int k = 0; k < g.n; k++) {
    const int pk = rl(g.pf, k);
    const bool mine = in && p == pk;
    const long long dl = mine ? (kind == K_COMPLETE ? -1 : kind == K_PLACE ? 1 : 0) : 0;
    if (mine) found = true;
    const long long inc = wscan_incl(dl);
    const long long cik = rl_i64(g.cnt, k) + inc;
    if (lane == k) tot_mine = rl_i64(inc, 63);
    if (in && cik < 1) bad = true;
    tocc += rl_f64(dvl, k) * (double)cik;
  }
  if (!found) bad = true;
  if (ballot(bad)) {
    for (int i = 0; i < m; i++) {
      const double occ = mkd(rlu(dlo(rc.occ), i), rlu(dhi(rc.occ), i));
      const long long dnet = mk64(rlu(lo32(rc.dnet), i), rlu(hi32(rc.dnet), i));
      const double dob = mkd(rlu(dlo(rc.dur), i), rlu(dhi(rc.dur), i));
      ws_fold<LW>(D, P, S, g, rl(kind, i), rl(w, i), rl(p, i), dnet, occ, rl(np, i), dob);
    }
    return;
  }
  const long long dn_inc = wscan_incl(in ? (long long)rc.dnet : 0);
  const double netocc_i = g.netocc + (double)dn_inc;
  tocc = tocc + netocc_i / (double)D.bandwidth;
  // check_idle_saturated's idle / saturated part for the record's worker
  const long long nt = in ? (long long)P.nthreads[w] : 1;
  const long long pp = np;
  const double avg = tocc / (double)D.total_nthreads;
  const bool paused = in && (P.wflags[w] & WF_PAUSED);
  bool idle = !paused && (pp < nt || rc.occ < (double)nt * avg / 2);
  bool sat = false;
  if (!idle && pp > nt && !paused) {
    const double pending = rc.occ * (double)(pp - nt) / (double)(pp * nt);
    sat = 0.4 < pending && pending > 1.9 * avg;
  }
  // the worker's last record in the batch decides its flags
  bool last = in;
  for (int j = 1; j < m; j++) {
    const int wj = rl(w, j);
    if (lane < j && w == wj) last = false;
  }
  int di = 0, ds = 0;
  if (last) {
    const uint8_t fo = P.wflags[w];
    const uint8_t fn = (fo & WF_PAUSED) | (idle ? WF_IDLE : 0) | (sat ? WF_SAT : 0);
    di = (idle ? 1 : 0) - ((fo & WF_IDLE) ? 1 : 0);
    ds = (sat ? 1 : 0) - ((fo & WF_SAT) ? 1 : 0);
    if (fo != fn) P.wflags[w] = fn;
  }
  g.n_idle += wsum(di);
  g.n_sat += wsum(ds);
  if (lane < g.n) g.cnt += tot_mine;
  g.netocc += (double)mk64(rlu(lo32(dn_inc), 63), rlu(hi32(dn_inc), 63));
}

template <bool LW>
__device__ __attribute__((always_inline)) void role_wlk(const Dev& D, SLds& L, const WPtr<LW>& P) {
  SCtl& S = L.c;
  const int lane = lane_id();
  WState g;
  while (true) {
    const long long wp = S.walk_pos;  // WLK (and a running global stimulus) write it
    const long long rl_ = vload(&S.rec_len);
    if (wp >= rl_) {
      if (vload(&S.stop)) break;
      __builtin_amdgcn_s_sleep(4);
      continue;
    }
    lds_fence();
    const int m = (int)min(rl_ - wp, (long long)64);
    SRec rc{};
    if (lane < m) rc = D.rlog[wp + lane];
    ws_load(S, g);
    const unsigned long long t0 = mclk();
    ws_fold_batch<LW>(D, P, S, g, rc, m);
    ws_store(S, g);
    lds_fence();
    if (lane == 0) {
      PROF(S.prof[4] += mclk() - t0);
      vstore(&S.walk_pos, wp + m);
      if (D.resident) S.t_role[6] = rclk();
    }
  }
}

// ====================================================================== sequencer
template <bool LW>
__device__ __attribute__((always_inline)) void snapshot(const Dev& D, SLds& L, const WPtr<LW>& P) {
  SCtl& S = L.c;
  const int lane = lane_id();
  const long long idx = S.rounds_nonempty;
  if (idx >= D.snap_cap) return;
  const DTab durv = (DTab)&S.wdur[0];
  for (int c0 = 0; c0 < D.W; c0 += 64) {
    const int c = min(c0 + lane, D.W - 1);
    const double o = occ_of<LW>(P, D, c, durv);
    if (c0 + lane < D.W) {
      const size_t k = (size_t)idx * D.W + c;
      D.snap_occ[k] = o;
      D.snap_nbytes[k] = P.nbytes[c];
      D.snap_nproc[k] = P.nproc[c];
      const bool itc = !(P.wflags[c] & WF_PAUSED) && (D.sat_inf || (int)P.cap[c] - P.nproc[c] > 0);
      D.snap_flags[k] = P.wflags[c] | (itc ? WF_ITC : 0);
    }
  }
  if (lane == 0) {
    D.snap_nplaced[idx] = (int32_t)(S.log_len - S.prev_placed);
    D.snap_nqueued[idx] = (int32_t)S.qlen;
    S.prev_placed = S.log_len;
  }
}

// every stimulus of the round is sequenced: count it, snapshot, open the next round.
// Returns true when the replay stops here.
// ---------------------------------------------------------- resident service mode
// The stream kernel stays launched between dgp_tasks_finished calls: the sequencer wave,
// once every stimulus of the request retired, publishes the answers (statuses, the log
// length, the new placements' task / worker) into the pinned mailbox, then polls it for the
// next request, answers its messages (svc::answer, Scheduler.stimulus_task_finished
// :5025-5092, as k_svc_append) and raises the stimulus end: the roles continue. Returns
// false when the kernel is to end (the host's stop, an error, or no request for a while).
__device__ __forceinline__ unsigned long long sys_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// exclusive prefix sum over the wave's lanes
__device__ __forceinline__ int wscan_excl(int v) {
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane_id() >= o) x += y;
  }
  return x - v;
}

// the compute-task message fields of placements [n0, n1) (_task_to_msg :3421-3450: who_has /
// nbytes of every dependency; dgp_msgs.h's rows) into the mailbox, 64 placements per step,
// each lane one placement; false when they exceed the mailbox's capacity (the host then asks
// dgp_task_messages' kernels)
__device__ __attribute__((noinline)) bool publish_messages(const Dev& D, svc::Mbox* mb, long long n0, long long n1) {
  const int lane = lane_id();
  int32_t* dptr = svc::mbox_m_dptr(mb);
  int32_t* dtask = svc::mbox_m_dtask(mb);
  int32_t* hptr = svc::mbox_m_hptr(mb);
  int32_t* hidx = svc::mbox_m_hidx(mb);
  int64_t* dnb = svc::mbox_m_dnb(mb);
  const long long cap = mb->md_cap;
  long long db = 0, hb = 0;
  for (long long k0 = 0; k0 < n1 - n0; k0 += 64) {
    const long long k = k0 + lane;
    const bool act = k < n1 - n0;
    const int t = act ? D.pl_task[n0 + k] : -1;
    int64_t a = 0, b = 0;
    int nh = 0;
    if (t >= 0 && t < D.N) {
      a = D.dep_ptr[t];
      b = D.dep_ptr[t + 1];
      for (int64_t q = a; q < b; q++) nh += msg::who_has_count(D, D.dep_idx[q]);
    }
    const int nd = (int)(b - a);
    const int sd = wscan_excl(nd), sh = wscan_excl(nh);
    const int td = wsum(nd), th = wsum(nh);
    if (db + td > cap || hb + th > cap) return false;
    if (act) {
      dptr[k] = (int32_t)(db + sd);
      long long e = db + sd, h = hb + sh;
      for (int64_t q = a; q < b; q++, e++) {
        const int d = D.dep_idx[q];
        dtask[e] = d;
        dnb[e] = D.cur_nbytes[d];
        hptr[e] = (int32_t)h;
        if (msg::multi_row(D, d)) {
          for (int w8 = 0; w8 < D.WB; w8++)
            for (unsigned long long m = D.holders[(size_t)d * D.WB + w8]; m; m &= m - 1) hidx[h++] = w8 * 64 + __builtin_ctzll(m);
        } else if (D.holder_of[d] >= 0) {
          hidx[h++] = D.holder_of[d];
        }
      }
    }
    db += td;
    hb += th;
  }
  if (lane == 0) {
    dptr[n1 - n0] = (int32_t)db;
    hptr[db] = (int32_t)hb;
  }
  return true;
}

__device__ __attribute__((noinline)) bool resident_serve(const Dev& D, SLds& L) {
  SCtl& S = L.c;
  const int lane = lane_id();
  svc::Mbox* mb = (svc::Mbox*)D.mbox;
  svc::Msg* msgs = svc::mbox_msgs(mb);
  int8_t* status = svc::mbox_status(mb);
  while (true) {
    if (S.req_off < S.req_n) {  // the next segment of the request in progress
      const long long len0 = *D.svc_len;
      long long len = len0, i = S.req_off;
      bool cut = false;
      while (i < S.req_n && !cut) {
        const long long k0 = i;
        svc::Msg m{};
        if (k0 + lane < S.req_n) m = msgs[k0 + lane];  // 64 messages across PCIe at once
        int8_t st = 0;
        const int kn = (int)min((long long)64, S.req_n - k0);
        int j = 0;
        for (; j < kn; j++) {
          svc::Msg mj;
          mj.task = rl(m.task, j);
          mj.worker = rl(m.worker, j);
          mj.run_id = rl_i64(m.run_id, j);
          mj.nbytes = rl_i64(m.nbytes, j);
          mj.start = rl_f64(m.start, j);
          mj.stop = rl_f64(m.stop, j);
          int8_t a = 0;
          bool take = false;
          if (lane == 0) take = svc::answer(D, mj, len0, len, a);
          if (__builtin_amdgcn_readfirstlane(take ? 1 : 0) == 0) {  // depends on this segment's stimuli
            cut = true;
            break;
          }
          len = rl_i64(len, 0);
          if (lane == j) st = (int8_t)rl((int)a, 0);
        }
        if (lane < j) status[k0 + lane] = st;
        i = k0 + j;
      }
      __threadfence();
      if (lane == 0) {
        *D.svc_len = len;
        S.req_off = i;
        S.stim_end = len;
        S.round_end = len;
        mb->t_app = rclk();
      }
      lds_fence();
      if (len > len0) return true;  // the roles run the new stimuli; back here when they retired
      continue;
    }
    if (S.req_seen != 0) {  // the request is answered: publish
      if (lane == 0) mb->t_ret = rclk();
      const long long n0 = S.req_pl0, n1 = S.log_len;
      const long long cap = mb->pl_cap;
      int32_t* pt = svc::mbox_pl_task(mb);
      int32_t* pw = svc::mbox_pl_worker(mb);
      if (n1 - n0 <= cap)
        for (long long k = lane; k < n1 - n0; k += 64) {
          pt[k] = D.pl_task[n0 + k];
          pw[k] = D.pl_worker[n0 + k];
        }
      const bool mok = __builtin_amdgcn_readfirstlane(mb->want_msgs) != 0 && n1 - n0 <= mb->mp_cap &&
                       publish_messages(D, mb, n0, n1);
      if (lane == 0) {
        mb->msg_from = mok ? n0 : -1;
        mb->pl_from = n1 - n0 <= cap ? n0 : -1;
        mb->n_placed = n1;
        mb->error = S.error;
        for (int k = 0; k < 7; k++) mb->t_role[k] = S.t_role[k];
        mb->t_pub = rclk();
      }
      __threadfence_system();
      if (lane == 0) __hip_atomic_store(&mb->done_seq, S.req_seen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (lane == 0) S.req_seen = 0;
      lds_fence();
    }
    // the next request, the host's stop, or an idle spell (then the kernel ends; the host
    // launches it again for the next request)
    const unsigned long long t0 = rclk();
    const unsigned long long last = sys_load(&mb->done_seq);
    unsigned long long rq = 0;
    while (true) {
      if (vload(&S.stop) || vload(&S.error)) return false;
      rq = sys_load(&mb->req_seq);
      if (rq != last) break;
      if (__hip_atomic_load(&mb->stop, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) return false;
      if (rclk() - t0 > 20000000ull) return false;  // 0.2 s without a request (100 MHz clock)
      __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) {
      mb->t_seen = rclk();
      S.req_seen = rq;
      S.req_n = (long long)__hip_atomic_load(&mb->n, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      S.req_off = 0;
      S.req_pl0 = S.log_len;
    }
    lds_fence();
  }
}

template <bool LW>
__device__ __attribute__((always_inline)) bool round_end_step(const Dev& D, SLds& L, const WPtr<LW>& P, long long& round_start) {
  SCtl& S = L.c;
  const int lane = lane_id();
  if (D.svc) {  // service mode: the launch ends with the stimulus log (no synthetic rounds)
    round_start = S.round_end;
    if (D.resident && resident_serve(D, L)) return false;  // the next request's stimuli
    if (lane == 0) vstore(&S.stop, 1);
    return true;
  }
  if (S.round_end > round_start) {
    if (lane == 0) S.rounds_nonempty++;
    wbar();
    if (S.snaps) {
      const unsigned long long t0 = rclk();
      while (vload(&S.walk_pos) != vload(&S.rec_len) || vload(&S.busy_exe) != 0) {
        if (vload(&S.stop)) return true;
        if (stalled_for(t0, rclk())) {
          serr(S, SERR_WATCHDOG, -2);
          return true;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      lds_fence();
      snapshot<LW>(D, L, P);
      __threadfence_block();
    }
    if (S.rounds_left > 0) {
      if (lane == 0) S.rounds_left--;
      wbar();
      if (S.rounds_left == 0) {
        round_start = S.round_end;
        if (lane == 0) vstore(&S.stop, 1);
        return true;
      }
    }
  }
  round_start = S.round_end;
  if (lane == 0) S.round_end = S.log_len;
  wbar();
  if (S.round_end == round_start) {  // the round just opened is empty: replay finished
    if (lane == 0) vstore(&S.stop, 1);
    return true;
  }
  if (lane == 0 && (S.snaps || S.rounds_left > 0)) vstore(&S.reg_limit, S.round_end);
  lds_fence();
  return false;
}

// The TaskState bookkeeping of a retired local completion (one lane per slot): the
// completed task (set_nbytes, processing_on, state; a dependent-less unwanted task is
// released at once) and the dependencies it released (:3309-3314, :2444-2505). Only
// exact / global stimuli and the host read these fields, and those run after every earlier
// slot has retired.
__device__ __forceinline__ void seq_bookkeeping(const Dev& D, long long r) {
  // the stimulus' descriptor row in the ring: PRE rewrites it only DR stimuli later, after
  // this one retired (its lead is bounded by seq_pos + DR)
  const uint4* row = D.desc + (size_t)(r & (DR - 1)) * NE;
  const uint4 e0 = row[0], e1 = row[1];
  const int t = (int)e0.x, w = (int)e0.y;
  const uint32_t flags = e0.w;
  const int64_t nbt = mk64(e1.x, e1.y);
  const int kt = e1.z & 0xff, nrel = (e1.z >> 8) & 0xff, grp_t = (int)e1.w;
  D.cur_nbytes[t] = nbt;
  D.proc_on[t] = -1;
  D.state[t] = (flags & F_SELFREL) ? S_RELEASED : S_MEMORY;
  if (flags & F_SELFREL) {
    atomicAdd((unsigned long long*)&D.g_relwait[grp_t], 1ull);
    D.holders[(size_t)t * D.WB + (w >> 6)] = 0;
  }
  for (int i = 0; i < nrel; i++) {
    const uint4 er = row[E_HDR + kt + i];
    const int d = (int)er.y, hd = (int)er.x;
    D.state[d] = S_RELEASED;
    D.holders[(size_t)d * D.WB + (hd >> 6)] = 0;
    atomicAdd((unsigned long long*)&D.g_relwait[D.group[d]], 1ull);
  }
}

template <bool LW>
__device__ __attribute__((always_inline)) void role_seq(const Dev& D, SLds& L, const WPtr<LW>& P, long long& round_start) {
  SCtl& S = L.c;
  const int lane = lane_id();
  unsigned long long t_sq = mclk(), t_idle = rclk();
  while (true) {
    if (vload(&S.stop)) break;
    const long long sp = S.seq_pos;
    const long long re = S.round_end;
    const long long r = sp + lane;
    const bool dn = r < re && vload(&L.rdone[r & (RS - 1)]) == r + 1;
    const unsigned long long b = ballot(dn);
    const int m = b == ~0ull ? 64 : (int)__builtin_ctzll(~b);  // ctz(0) is undefined
    if (m == 0) {
      if (sp == re) {
        if (round_end_step<LW>(D, L, P, round_start)) break;
        t_idle = rclk();
        continue;
      }
      const unsigned long long nw = mclk();
      if (stalled_for(t_idle, rclk())) {
        serr(S, SERR_WATCHDOG, (int)sp);
        break;
      }
      PROF(if (lane == 0) S.prof[30] += nw - t_sq);  // 30: sequencer waiting for the oldest slot
      t_sq = nw;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    lds_fence();
    {  // invariants of the control block (cheap; a violation names the field)
      const long long rp = vload(&S.reg_pos);
      const int be = vload(&S.busy_exe), gp = vload(&S.global_pending);
      int bad = 0;
      if (rp < sp || rp > sp + RS) bad = 1;
      if (be < 0 || be > 16) bad = 2;
      if (gp < 0 || gp > 1) bad = 3;
      if (S.qlen < 0 || S.qhead < 0) bad = 4;
      if (bad) {
        serr(S, SERR_INV, bad * 100000000 + (int)sp);
        break;
      }
    }
    const unsigned long long t0 = mclk();
    const int q = (int)(r & (RS - 1));  // retire-ring entry and staging rows of stimulus r
    int npl = 0, nrec = 0, npop = 0;
    bool direct = false;
    if (lane < m) {
      const RMeta me = L.rmeta[q];
      npl = me.npl;
      nrec = me.nrec;
      npop = me.npops;
      direct = me.direct != 0;
    }
    if (ballot(lane < m && (npl < 0 || nrec < 0 || npop < 0 || npop > npl || (!direct && (npl > PLC || nrec > PLC))))) {
      serr(S, SERR_INV, 500000000 + (int)sp);
      break;
    }
    int ipl = npl, irc = nrec, ipo = npop;
    for (int o = 1; o < 64; o <<= 1) {
      const int a = __shfl_up(ipl, o), b2 = __shfl_up(irc, o), c2 = __shfl_up(ipo, o);
      if (lane >= o) {
        ipl += a;
        irc += b2;
        ipo += c2;
      }
    }
    const int tpl = rl(ipl, 63), trc = rl(irc, 63), tpo = rl(ipo, 63);
    const long long lb = S.log_len + (ipl - npl), rb = S.rec_len + (irc - nrec), qb = S.qhead + (ipo - npop);
    // capacity first: nothing is copied past the record log (rlog_cap = 2N + 4096 covers one
    // K_COMPLETE per completion and one K_PLACE per placement, the only record kinds)
    if (S.rec_len + trc > D.rlog_cap || S.log_len + tpl > D.pl_cap) {
      serr(S, SERR_REC, (int)sp);
      break;
    }
    if (lane < m && !direct) {
      const size_t st0 = (size_t)q * PLC;
      int popk = 0;
      for (int j = 0; j < npl; j++) {
        int task = D.s2_task[st0 + j];
        const int w = D.s2_worker[st0 + j];
        const long long pos = lb + j;
        if (task < 0) {  // a queued task taken by the stimulus' refill: HeapSet order
          task = D.qarr[qb + popk++];
          D.state[task] = S_PROCESSING;
          D.proc_on[task] = w;
        } else {  // a frontier placement (waiting -> processing, :2313-2336): TaskState and the
                  // group's released + waiting count, off the executors' path (only exact /
                  // global stimuli and the host read them, after this retirement)
          D.state[task] = S_PROCESSING;
          D.proc_on[task] = w;
          atomicAdd((unsigned long long*)&D.g_relwait[D.group[task]], (unsigned long long)-1ll);
        }
        D.pl_task[pos] = task;
        D.pl_worker[pos] = w;
        D.pl_comm[pos] = D.s2_comm[st0 + j];
        D.pl_start[pos] = D.s2_start[st0 + j];
        D.pl_wsnbytes[pos] = D.s2_wsnb[st0 + j];
        D.pl_route[pos] = D.s2_route[st0 + j];
        D.run_id[task] = (int32_t)pos;
        D.holder_of[task] = w;
      }
      for (int j = 0; j < nrec; j++) D.rlog[rb + j] = D.srec[st0 + j];
      seq_bookkeeping(D, r);
    }
    __threadfence_block();
    if (lane == 0) {
      S.log_len += tpl;
      S.rec_len += trc;
      S.qhead += tpo;
      S.qlen -= tpo;
      S.n_tasks += tpl;
      PROF(S.prof[0] += mclk() - t0);
      PROF(S.prof[8] += 1);
    }
    lds_fence();
    if (lane == 0) {
      vstore(&S.seq_pos, sp + m);
      if (D.resident) S.t_role[5] = rclk();
      if (DGP_TRACE) {
        const unsigned long long tn = __builtin_amdgcn_s_memtime();
        if (TRL) for (int i = 0; i < m; i++) trace_at(D, sp + i, 6, tn);
      }

    }
    t_idle = rclk();
    t_sq = mclk();
  }
}

// ======================================================================= builder
// completions [a, e) (one per lane): the waiting_on / waiters decrements. A row wider than
// BLD_NARROW (a completion with many dependents or dependencies: the shuffle barrier's
// 66,666; a task whose fan-in / fan-out max is wide) would be one lane's serial chain of
// dependent loads, so it becomes a job the whole wave takes 64 entries at a time.
constexpr int BLD_NARROW = 32;
constexpr int BLD_JOBS = 256;
enum : int { BJ_COMPLETE = 0, BJ_FRMARK = 1, BJ_RELMARK = 2 };

__device__ __forceinline__ bool bld_push(SLds& L, int kind, int x) {
  const int j = atomicAdd(&L.bld_njobs, 1);
  if (j >= BLD_JOBS) return false;  // full: the caller does it itself
  L.bld_jobs[j] = (kind << 28) | x;
  return true;
}
// the stimulus that empties x's waiting_on: its dependency completed last (one lane)
__device__ __forceinline__ int fr_of(const Dev& D, int x) {
  int s = -1;
  for (int64_t q = D.dep_ptr[x]; q < D.dep_ptr[x + 1]; q++) s = max(s, D.cseq[D.dep_idx[q]]);
  return s;
}
// the stimulus that empties d's waiters: its dependent completed last (one lane)
__device__ __forceinline__ int rel_of(const Dev& D, int d) {
  int s = -1;
  for (int64_t q = D.dpt_ptr[d]; q < D.dpt_ptr[d + 1]; q++) s = max(s, D.cseq[D.dpt_idx[q]]);
  return s;
}
// waiting_on.discard for dependent x of a completion (:3298-3307) and waiters.discard ->
// release for dependency d (:3309-3314); the lane that empties the set marks the stimulus
__device__ __forceinline__ void bld_dec_dependent(const Dev& D, SLds& L, int x) {
  if (atomicSub(&D.remaining[x], 1) == 1) {
    if (D.dep_ptr[x + 1] - D.dep_ptr[x] <= BLD_NARROW || !bld_push(L, BJ_FRMARK, x)) D.fr_mark[x] = fr_of(D, x);
  }
}
__device__ __forceinline__ void bld_dec_dependency(const Dev& D, SLds& L, int d) {
  if (atomicSub(&D.waiters[d], 1) == 1 && !(D.tflags[d] & TF_WANTED)) {
    if (D.dpt_ptr[d + 1] - D.dpt_ptr[d] <= BLD_NARROW || !bld_push(L, BJ_RELMARK, d)) D.rel_mark[d] = rel_of(D, d);
  }
}

__device__ __attribute__((always_inline)) void bld_range(const Dev& D, SLds& L, long long a, long long e) {
  const int lane = lane_id();
  const long long r = a + lane;
  if (r < e) {
    const int t = D.stim_task[r];
    const int w = D.stim_worker[r];
    // the replica this completion creates (who_has, :3148)
    atomicOr(&D.holders[(size_t)t * D.WB + (w >> 6)], 1ull << (w & 63));
    const int64_t f0 = D.dpt_ptr[t], f1 = D.dpt_ptr[t + 1], k0 = D.dep_ptr[t], k1 = D.dep_ptr[t + 1];
    if ((f1 - f0 > BLD_NARROW || k1 - k0 > BLD_NARROW) && bld_push(L, BJ_COMPLETE, t)) {
      // the wave takes it below
    } else {
      for (int64_t k = f0; k < f1; k++) bld_dec_dependent(D, L, D.dpt_idx[k]);
      for (int64_t k = k0; k < k1; k++) bld_dec_dependency(D, L, D.dep_idx[k]);
    }
  }
  // the wide rows, 64 entries at a time (jobs may add jobs: a wide completion empties a
  // wide task)
  lds_fence();
  int done = 0;
  while (true) {
    const int nj = min(vload(&L.bld_njobs), BLD_JOBS);
    if (done >= nj) break;
    for (int j = done; j < nj; j++) {
      const int code = L.bld_jobs[j];
      const int kind = code >> 28, x = code & 0x0fffffff;
      if (kind == BJ_COMPLETE) {
        const int64_t f0 = D.dpt_ptr[x], f1 = D.dpt_ptr[x + 1], k0 = D.dep_ptr[x], k1 = D.dep_ptr[x + 1];
        for (int64_t k = f0 + lane; k < f1; k += 64) bld_dec_dependent(D, L, D.dpt_idx[k]);
        for (int64_t k = k0 + lane; k < k1; k += 64) bld_dec_dependency(D, L, D.dep_idx[k]);
      } else {
        const bool fr = kind == BJ_FRMARK;
        const int64_t q0 = fr ? D.dep_ptr[x] : D.dpt_ptr[x], q1 = fr ? D.dep_ptr[x + 1] : D.dpt_ptr[x + 1];
        int m = -1;
        for (int64_t q = q0 + lane; q < q1; q += 64) m = max(m, D.cseq[fr ? D.dep_idx[q] : D.dpt_idx[q]]);
        m = wmax(m);
        if (lane == 0) (fr ? D.fr_mark : D.rel_mark)[x] = m;
      }
      lds_fence();
    }
    done = nj;
  }
  wbar();
  if (lane == 0) L.bld_njobs = 0;
  lds_fence();
}

// ==================================================================== prefetcher
// descriptor of stimulus r (one lane): see E_HDR for the header layout
__device__ __attribute__((always_inline)) void build_desc_seq(const Dev& D, SLds& L, long long r, int& p_out, double& dobs_out) {
  uint4* E = D.desc + (size_t)(r & (DR - 1)) * NE;
  // the distinct workers the stimulus touches, in first-touch order (lane-private LDS list)
  auto scr = L.pre_scr[lane_id()];
  int nt = 0;
  bool tbad = false;
  // service events the local path does not model make the stimulus global (exe_global):
  // a paused worker (not in running), a replica set beyond holder_of, a long-running task
  bool evg = false;
  auto touch = [&](int c, bool cand) -> int {  // -> its index in the touch list (-1: none)
    if (c < 0 || c >= D.W) {
      tbad = true;
      return -1;
    }
    if ((D.evf & EVF_PAUSED) && (D.w_flags[c] & WF_PAUSED)) evg = true;
    for (int i = 0; i < nt && i < TMAX; i++)
      if ((scr[i] & T_W) == c) {
        if (cand) scr[i] |= (uint16_t)T_CAND;
        return i;
      }
    if (nt < TMAX) scr[nt] = (uint16_t)(c | (cand ? T_CAND : 0));
    return nt++ < TMAX ? nt - 1 : -1;
  };
  const int t = D.stim_task[r];
  const int w = D.stim_worker[r];
  const int p = D.prefix[t];
  const int g = D.group[t];
  const uint8_t tf = D.tflags[t];
  const int64_t nbt = nbv(D, D.res_nbytes[t]);
  const double dobs = D.res_stop[t] - D.res_start[t];
  const int64_t k0 = D.dep_ptr[t], k1 = D.dep_ptr[t + 1];
  const int64_t f0 = D.dpt_ptr[t], f1 = D.dpt_ptr[t + 1];
  const int kt = (int)(k1 - k0);
  uint32_t flags = 0;
  if (f1 == f0 && !(tf & TF_WANTED)) flags |= F_SELFREL;
  if ((D.evf & EVF_LR) && (D.tdyn[t] & TD_LR)) evg = true;
  if (kt > KT_MAX) {
    flags |= F_GLOBAL;
    PROF(atomicAdd(&L.c.prof[20], 1ull));  // diagnostics: why stimuli run global
  }
  int n = E_HDR, nrel = 0, nf = 0, sumkx = 0;
  touch(w, false);
  int h_dep0 = -1;  // holder of the first dependency
  if (!(flags & F_GLOBAL)) {
    for (int64_t k = k0; k < k1; k++) {
      const int d = D.dep_idx[k];
      const int64_t nb = nbv(D, D.res_nbytes[d]);
      const int hd = D.holder_of[d];
      if (k == k0) h_dep0 = hd;
      if ((D.evf & EVF_MULTI) && (D.tdyn[d] & TD_MULTI)) evg = true;
      E[n++] = make_uint4((unsigned)d, (unsigned)hd, lo32(nb), hi32(nb));
    }
    for (int64_t k = k0; k < k1; k++) {
      const int d = D.dep_idx[k];
      if (D.rel_mark[d] != (int)r) continue;
      if (n >= NE) {
        flags |= F_GLOBAL;
        break;
      }
      const int64_t nb = nbv(D, D.res_nbytes[d]);
      const int hd = D.holder_of[d];
      touch(hd, false);
      E[n++] = make_uint4((unsigned)hd, (unsigned)d, lo32(nb), hi32(nb));
      nrel++;
    }
  }
  // dependents in ascending priority = frontier order; a global stimulus walks its frontier
  // itself (exe_global), so the walk stops there
  for (int64_t k = f0; k < f1 && !(flags & F_GLOBAL); k++) {
    const int x = D.dpt_idx[k];
    if (D.fr_mark[x] != (int)r) continue;
    nf++;
    const int64_t x0 = D.dep_ptr[x], x1 = D.dep_ptr[x + 1];
    const int kx = (int)(x1 - x0);
    if ((D.tflags[x] & TF_ROOTISH) || kx > KX_MAX || n + 1 + kx > NE) {
      if (!(flags & F_GLOBAL)) PROF(atomicAdd(&L.c.prof[(D.tflags[x] & TF_ROOTISH) ? 16 : 21], 1ull));
      flags |= F_GLOBAL;
      continue;
    }
    // a restricted task (f1): decide_worker's candidates (:8575-8586) resolved here —
    // holders & valid; none: the valid set; valid empty: loose -> the holders, else
    // no-worker (global). They follow the dependency entries; the holders are not touched
    const bool rx = restricted_nonrootish(D, x);
    int cw[RC_MAX];
    int nc = 0;
    if (rx) {
      for (int64_t q = x0; q < x1 && nc >= 0; q++) {
        const int hd = D.holder_of[D.dep_idx[q]];
        bool dup = false;
        for (int i = 0; i < nc; i++) dup = dup || cw[i] == hd;
        if (!dup && hd >= 0 && hd < D.W && restr_has(D, x, hd)) cw[nc++] = hd;
      }
      const RRow rr = restr_row(D, x);
      const int64_t r0 = rr.r0, r1 = rr.r1;
      if (nc == 0 && r1 > r0) {
        if (r1 - r0 > RC_MAX) nc = -1;
        else for (int64_t i = r0; i < r1; i++) cw[nc++] = rr.idx[i];
      } else if (nc == 0) {
        if (!(D.restr_flags[x] & RF_LOOSE)) nc = -1;  // no-worker
        else for (int64_t q = x0; q < x1; q++) {       // decide_worker without restrictions
          const int hd = D.holder_of[D.dep_idx[q]];
          bool dup = false;
          for (int i = 0; i < nc; i++) dup = dup || cw[i] == hd;
          if (!dup) cw[nc++] = hd;
        }
      }
      if (nc < 0 || n + 1 + kx + nc > NE) {
        flags |= F_GLOBAL;
        continue;
      }
    }
    const int nx = n++;  // the task's entry, written below with its candidates' touch mask
    sumkx += kx;
    // decide_worker's candidates (:8571-8574) are the dependencies' holders: their touch
    // indices, the mask the executor's argmin takes
    int tix[KX_MAX];
#pragma unroll
    for (int q = 0; q < KX_MAX; q++) {
      tix[q] = -1;
      if (q < kx) {
        const int d = D.dep_idx[x0 + q];
        const int64_t nb = nbv(D, D.res_nbytes[d]);
        const int hd = D.holder_of[d];
        if ((D.evf & EVF_MULTI) && (D.tdyn[d] & TD_MULTI)) evg = true;
        if (!rx) tix[q] = touch(hd, true);
        E[n++] = make_uint4((unsigned)d, (unsigned)hd, lo32(nb), hi32(nb));
      }
    }
    uint32_t cmask = 0;  // touch indices (< 32) of the candidates
    if (!rx) {
#pragma unroll
      for (int q = 0; q < KX_MAX; q++) {
        const int i = tix[q];
        if (q < kx && i >= 0 && i < 32) cmask |= 1u << i;
      }
    }
    E[nx] = make_uint4((unsigned)x, (unsigned)D.prefix[x], (unsigned)(kx | (nc << 8) | (rx ? 1 << 16 : 0)), cmask);
    for (int i = 0; i < nc; i++) {
      touch(cw[i], true);
      E[n++] = make_uint4((unsigned)cw[i], 0u, 0u, 0u);
    }
  }
  if (!(flags & F_GLOBAL) && (nf > 255 || nt > TMAX || nf + (D.sat_inf ? 0 : D.w_cap[w]) + 1 > PLC))
    PROF(atomicAdd(&L.c.prof[22], 1ull));
  if (nf > 255 || nt > TMAX) flags |= F_GLOBAL;
  if (nf + (D.sat_inf ? 0 : D.w_cap[w]) + 1 > PLC) flags |= F_GLOBAL;  // staging room for the refill
  if (tbad) flags |= F_GLOBAL | F_BADTOUCH;
  if (evg) flags |= F_GLOBAL;
  if (!(flags & F_GLOBAL) && nt == 1 && nf == 0 && kt <= 1 && nrel <= 1 &&
      (kt == 0 || h_dep0 >= 0) && D.P <= PD)  // a run shares the head's descriptor durations
    flags |= F_SIMPLE;
  if (flags & F_GLOBAL) nt = 0;
  int32_t* T = D.touch_ring + (size_t)(r & (DR - 1)) * TMAX;
  for (int i = 0; i < nt; i++) T[i] = scr[i];
  E[0] = make_uint4((unsigned)t, (unsigned)w, (unsigned)p, flags);
  E[1] = make_uint4(lo32(nbt), hi32(nbt),
                    (unsigned)(min(kt, 255) | (nrel << 8) | (min(nf, 255) << 16) | (n << 24)), (unsigned)g);
  E[2] = make_uint4(dlo(dobs), dhi(dobs), (unsigned)nt, (unsigned)sumkx);  // sumkx: needs entries it may add
  D.thdr[r & (DR - 1)] = make_uint2(flags, (unsigned)nt);
  p_out = p;
  dobs_out = dobs;
}

// The gathered form of build_desc: every load of one dependency level is issued before any
// store (a store to the ring would order each later load behind it), 8 entries at a time, so
// a lane's descriptor costs a handful of memory round trips -- the stimulus, its task, the
// dependency ids, their fields (holders, sizes, release marks), the dependent ids and their
// frontier marks, then per frontier task its fields, its dependencies' ids and fields --
// instead of one or two per entry. PRE's batch is as slow as its slowest lane, so every
// size takes this path (a completion with many dependents costs one more pair of round trips
// per 8 of them). The descriptor and the touch list come out exactly as
// build_desc_seq writes them. false (nothing written): the graph has restrictions (their
// resolved candidates stay with build_desc_seq).
constexpr int GC = 8;  // entries gathered per round trip
__device__ __attribute__((always_inline)) bool build_desc_g(const Dev& D, SLds& L, long long r, int& p_out, double& dobs_out) {
  if (D.restr_flags) return false;
  const int t = D.stim_task[r];
  const int w = D.stim_worker[r];
  // ---- the completing task (one round trip)
  const int p = D.prefix[t];
  const int g = D.group[t];
  const uint8_t tf = D.tflags[t];
  const int64_t nbraw = D.res_nbytes[t];
  const double stop = D.res_stop[t], start = D.res_start[t];
  const int64_t k0 = D.dep_ptr[t], k1 = D.dep_ptr[t + 1];
  const int64_t f0 = D.dpt_ptr[t], f1 = D.dpt_ptr[t + 1];
  const uint8_t tdt = (D.evf & EVF_LR) ? D.tdyn[t] : 0;
  const int capw = D.sat_inf ? 0 : D.w_cap[w];
  const int kt = (int)(k1 - k0);
  uint4* E = D.desc + (size_t)(r & (DR - 1)) * NE;
  auto scr = L.pre_scr[lane_id()];
  int nt = 0;
  bool tbad = false, evg = false;
  auto touch = [&](int c, bool cand) -> int {  // -> its index in the touch list (-1: none)
    if (c < 0 || c >= D.W) {
      tbad = true;
      return -1;
    }
    if ((D.evf & EVF_PAUSED) && (D.w_flags[c] & WF_PAUSED)) evg = true;
    for (int i = 0; i < nt && i < TMAX; i++)
      if ((scr[i] & T_W) == c) {
        if (cand) scr[i] |= (uint16_t)T_CAND;
        return i;
      }
    if (nt < TMAX) scr[nt] = (uint16_t)(c | (cand ? T_CAND : 0));
    return nt++ < TMAX ? nt - 1 : -1;
  };
  const int64_t nbt = nbv(D, nbraw);
  const double dobs = stop - start;
  uint32_t flags = 0;
  if (f1 == f0 && !(tf & TF_WANTED)) flags |= F_SELFREL;
  if (tdt & TD_LR) evg = true;
  if (kt > KT_MAX) flags |= F_GLOBAL;
  int n = E_HDR, nrel = 0, nf = 0, sumkx = 0;
  int h_dep0 = -1;
  touch(w, false);
  uint32_t relm = 0;  // dependencies (< KT_MAX) released by this completion
  if (!(flags & F_GLOBAL)) {
    // ---- dependencies: ids, then fields, GC at a time; their entries in order
    for (int c0 = 0; c0 < kt; c0 += GC) {
      int dq[GC];
#pragma unroll
      for (int q = 0; q < GC; q++) dq[q] = c0 + q < kt ? D.dep_idx[k0 + c0 + q] : 0;
      int64_t nbq[GC];
      int hq[GC], rmq[GC];
      bool mq[GC];
#pragma unroll
      for (int q = 0; q < GC; q++) {
        nbq[q] = 0;
        hq[q] = rmq[q] = -1;
        mq[q] = false;
        if (c0 + q < kt) {
          nbq[q] = nbv(D, D.res_nbytes[dq[q]]);
          hq[q] = D.holder_of[dq[q]];
          rmq[q] = D.rel_mark[dq[q]];
          mq[q] = (D.evf & EVF_MULTI) && (D.tdyn[dq[q]] & TD_MULTI);
        }
      }
#pragma unroll
      for (int q = 0; q < GC; q++)
        if (c0 + q < kt) {
          if (c0 + q == 0) h_dep0 = hq[q];
          if (mq[q]) evg = true;
          if (rmq[q] == (int)r) relm |= 1u << (c0 + q);
          E[n++] = make_uint4((unsigned)dq[q], (unsigned)hq[q], lo32(nbq[q]), hi32(nbq[q]));
        }
    }
    // ---- the releases (their dependency entries read back, one round trip)
    for (uint32_t m = relm; m && !(flags & F_GLOBAL); m &= m - 1) {
      if (n >= NE) {
        flags |= F_GLOBAL;
        break;
      }
      const uint4 er = E[E_HDR + __builtin_ctz(m)];
      touch((int)er.y, false);
      E[n++] = make_uint4(er.y, er.x, er.z, er.w);
      nrel++;
    }
  }
  // ---- dependents in ascending priority = frontier order (a global stimulus stops the walk)
  const int nd = (int)(f1 - f0);
  for (int c0 = 0; c0 < nd && !(flags & F_GLOBAL); c0 += GC) {
    int xq[GC];
#pragma unroll
    for (int q = 0; q < GC; q++) xq[q] = c0 + q < nd ? D.dpt_idx[f0 + c0 + q] : 0;
    int frq[GC];
#pragma unroll
    for (int q = 0; q < GC; q++) frq[q] = c0 + q < nd ? D.fr_mark[xq[q]] : -1;
    // the frontier tasks of this chunk: their fields at once
    uint8_t ftf[GC];
    int64_t fx0[GC];
    int fkx[GC], fpx[GC];
#pragma unroll
    for (int q = 0; q < GC; q++) {
      ftf[q] = 0;
      fx0[q] = 0;
      fkx[q] = 0;
      fpx[q] = 0;
      if (frq[q] == (int)r) {
        const int x = xq[q];
        ftf[q] = D.tflags[x];
        fx0[q] = D.dep_ptr[x];
        fkx[q] = (int)(D.dep_ptr[x + 1] - fx0[q]);
        fpx[q] = D.prefix[x];
      }
    }
    uint32_t fm = 0;  // the chunk's frontier tasks
#pragma unroll
    for (int q = 0; q < GC; q++) fm |= frq[q] == (int)r ? 1u << q : 0u;
    static_assert(GC == 8, "DGP_SEL8");
#define DGP_SEL8(a, q) \
  ((q) == 0 ? a[0] : (q) == 1 ? a[1] : (q) == 2 ? a[2] : (q) == 3 ? a[3] : (q) == 4 ? a[4] : (q) == 5 ? a[5] : (q) == 6 ? a[6] : a[7])
#pragma unroll 1
    for (; fm && !(flags & F_GLOBAL); fm &= fm - 1) {
      const int q = __builtin_ctz(fm);  // (lane-varying: selected without indexing the arrays)
      nf++;
      const int x = DGP_SEL8(xq, q), kx = DGP_SEL8(fkx, q);
      const uint8_t ftq = DGP_SEL8(ftf, q);
      const int64_t fxq = DGP_SEL8(fx0, q);
      const int fpq = DGP_SEL8(fpx, q);
      if ((ftq & TF_ROOTISH) || kx > KX_MAX || n + 1 + kx > NE) {
        flags |= F_GLOBAL;
        continue;
      }
      // its dependencies: ids, then fields
      int dx[KX_MAX];
#pragma unroll
      for (int i = 0; i < KX_MAX; i++) dx[i] = i < kx ? D.dep_idx[fxq + i] : 0;
      int64_t nbx[KX_MAX];
      int hx[KX_MAX];
#pragma unroll
      for (int i = 0; i < KX_MAX; i++) {
        nbx[i] = 0;
        hx[i] = -1;
        if (i < kx) {
          nbx[i] = nbv(D, D.res_nbytes[dx[i]]);
          hx[i] = D.holder_of[dx[i]];
          if ((D.evf & EVF_MULTI) && (D.tdyn[dx[i]] & TD_MULTI)) evg = true;
        }
      }
      const int nx = n++;
      sumkx += kx;
      // decide_worker's candidates (:8571-8574) are the dependencies' holders: their touch
      // indices, the mask the executor's argmin takes
      int tix[KX_MAX];
#pragma unroll
      for (int i = 0; i < KX_MAX; i++) {
        tix[i] = -1;
        if (i < kx) {
          tix[i] = touch(hx[i], true);
          E[n++] = make_uint4((unsigned)dx[i], (unsigned)hx[i], lo32(nbx[i]), hi32(nbx[i]));
        }
      }
      uint32_t cmask = 0;  // touch indices (< 32) of the candidates
#pragma unroll
      for (int i = 0; i < KX_MAX; i++) {
        const int ti = tix[i];
        if (i < kx && ti >= 0 && ti < 32) cmask |= 1u << ti;
      }
      E[nx] = make_uint4((unsigned)x, (unsigned)fpq, (unsigned)kx, cmask);
    }
#undef DGP_SEL8
  }
  if (nf > 255 || nt > TMAX) flags |= F_GLOBAL;
  if (nf + capw + 1 > PLC) flags |= F_GLOBAL;  // staging room for the refill
  if (tbad) flags |= F_GLOBAL | F_BADTOUCH;
  if (evg) flags |= F_GLOBAL;
  if (!(flags & F_GLOBAL) && nt == 1 && nf == 0 && kt <= 1 && nrel <= 1 && (kt == 0 || h_dep0 >= 0) && D.P <= PD)
    flags |= F_SIMPLE;  // a run shares the head's descriptor durations
  if (flags & F_GLOBAL) nt = 0;
  int32_t* T = D.touch_ring + (size_t)(r & (DR - 1)) * TMAX;
  for (int i = 0; i < nt; i++) T[i] = scr[i];
  E[0] = make_uint4((unsigned)t, (unsigned)w, (unsigned)p, flags);
  E[1] = make_uint4(lo32(nbt), hi32(nbt),
                    (unsigned)(min(kt, 255) | (nrel << 8) | (min(nf, 255) << 16) | (n << 24)), (unsigned)g);
  E[2] = make_uint4(dlo(dobs), dhi(dobs), (unsigned)nt, (unsigned)sumkx);
  D.thdr[r & (DR - 1)] = make_uint2(flags, (unsigned)nt);
  p_out = p;
  dobs_out = dobs;
  return true;
}
struct DescOut {
  int ok, p;
  double dobs;
};
// out of line: each form gets its own register allocation (inlined together they spilled)
__device__ __attribute__((noinline)) DescOut build_desc_g_entry(long long r) {
  DescOut o{0, 0, 0.0};
  o.ok = build_desc_g(c_dev, st_L(), r, o.p, o.dobs) ? 1 : 0;
  return o;
}
__device__ __attribute__((noinline)) DescOut build_desc_seq_entry(long long r) {
  DescOut o{1, 0, 0.0};
  build_desc_seq(c_dev, st_L(), r, o.p, o.dobs);
  return o;
}
__device__ __forceinline__ void build_desc(const Dev& D, SLds& L, long long r, int& p_out, double& dobs_out) {
  DescOut o{0, 0, 0.0};
  o = build_desc_g_entry(r);
  if (!o.ok) o = build_desc_seq_entry(r);
  p_out = o.p;
  dobs_out = o.dobs;
}

// ========================================================== builder / prefetcher
// One wave each, in the engine workgroup (every hand-off stays on this CU: workgroup-scope
// LDS positions, no cross-CU visibility to manage). Each takes the next range of up to 64
// stimuli (one per lane) below its bound: BLD below the log length, PRE below BLD and
// the descriptor ring.
template <int KIND>  // 0 BLD, 1 PRE
__device__ __attribute__((always_inline)) void role_stage(const Dev& D, SLds& L) {
  SCtl& S = L.c;
  const int lane = lane_id();
  // PRE: lane p holds TaskPrefix.duration_average of prefix p as of pre_pos, and its
  // max_exec_time (heartbeats change it only between launches): no load in the fold loop,
  // whose stores would otherwise each be waited for before the next iteration's load
  double dur = (KIND == 1 && lane < PX && lane < D.P) ? D.pdur_pre[lane] : -1.0;
  const double pmx = (KIND == 1 && lane < PX && lane < D.P) ? D.pmaxexec[lane] : -1.0;
  auto resolve = [&](double d) { return d < 0 ? (pmx > 0 ? 2 * pmx : D.unknown_duration) : d; };  // :1892-1899
  while (true) {
    if (vload(&S.stop)) break;
    const long long a = KIND == 0 ? S.bld_pos : S.pre_pos;
    // BLD: completions up to the placement log (replay: stimulus r completes placement r)
    // or the stimulus log (service); PRE: what BLD has built, at most pre_lead ahead of SEQ
    const long long hi = KIND == 0 ? (D.svc ? vload(&S.stim_end) : vload(&S.log_len))
                                   : min(vload(&S.bld_pos), vload(&S.seq_pos) + D.pre_lead);
    const long long e = min(a + 64, hi);
    if (e <= a) {
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    lds_fence();
    const unsigned long long t0 = mclk();
    if (KIND == 0) {
      bld_range(D, L, a, e);
    } else {
      const long long r = a + lane;
      int pl = 0;
      double dl = 0.0;
      if (r < e) build_desc(D, L, r, pl, dl);
      // TaskPrefix.add_duration (:977-985) in stimulus order; each descriptor carries the
      // resolved durations (_calc_occupancy :1892-1899) after its own completion, entries 3..6
      const int m = (int)(e - a);
      for (int i = 0; i < m; i++) {
        const int pi = rl(pl, i);
        const double di = mkd(rlu(dlo(dl), i), rlu(dhi(dl), i));
        if (lane == pi && di == di) dur = dur < 0 ? di : 0.5 * di + 0.5 * dur;  // NaN: no compute interval
        if (D.P <= PD) {
          if (lane < PD) ((double*)(D.desc + (size_t)((a + i) & (DR - 1)) * NE + 3))[lane] = lane < D.P ? resolve(dur) : -1.0;
        } else if (lane < D.P) {
          D.dring[(size_t)((a + i) & (DR - 1)) * PX + lane] = resolve(dur);
        }
      }
    }
    __threadfence_block();
    wbar();
    if (lane == 0) {
      PROF(S.prof[KIND == 0 ? 1 : 2] += mclk() - t0);
      PROF(S.prof[KIND == 0 ? 6 : 7] += 1);
      vstore(KIND == 0 ? &S.bld_pos : &S.pre_pos, e);
      if (D.resident) S.t_role[KIND] = rclk();
    }
  }
  if (KIND == 1 && lane < PX && lane < D.P) D.pdur_pre[lane] = dur;
}

// ===================================================================== registrar
// In stimulus order: the slot flags, the distinct touched workers, then registration (slot
// bit into each touched worker's mask; predecessor count = the in-flight bits already
// there). The descriptor itself stays in the global ring (the executors read it there) and
// PRE has already resolved its durations, so a batch of up to RB stimuli moves only the
// touch lists and the per-slot words (lane b = stimulus b). Phase A prepares every slot of
// the batch; phase B registers them. The mask atomics of phase B are issued back to back:
// one wave's LDS operations execute in order, so stimulus b sees the bits of b-1 exactly as
// if they were registered one at a time.

template <bool LW>
__device__ __attribute__((always_inline)) void role_reg(const Dev& D, SLds& L, const WPtr<LW>& P) {
  SCtl& S = L.c;
  const int lane = lane_id();
  constexpr int RB = DGP_RB;
  long long pre = 0;  // cached PRE watermark: re-read only when exhausted
  unsigned long long t_poll = mclk();
  int TB[RB];   // touch lists of the batch: lane i = touched worker i of stimulus r0 + b
  uint2 HB;     // lane b: (flags, touched-worker count) of stimulus r0 + b (PRE's row header)
  long long eb_first = -1;
  int eb_n = 0;
  int prev_simple_w = -1;  // the last registered stimulus' worker if it was F_SIMPLE, else -1
  auto fetch = [&](long long r1, int n1) {  // the rows of stimuli [r1, r1 + n1)
#pragma unroll
    for (int b = 0; b < RB; b++)
      TB[b] = (lane < TMAX && b < n1) ? D.touch_ring[(size_t)((r1 + b) & (DR - 1)) * TMAX + lane] : -1;
    HB = lane < n1 ? D.thdr[(r1 + lane) & (DR - 1)] : make_uint2(0, 0);
    eb_first = r1;
    eb_n = n1;
  };
  while (true) {
    if (vload(&S.stop)) break;
    const long long r0 = S.reg_pos;
    if (r0 >= pre) pre = vload(&S.pre_pos);
    const long long wl = vload(&S.seq_pos) + RS;  // retire-ring capacity
    const SMask fm = vload(&S.freem);              // free slots (only this wave takes them)
    const long long lim = min(min(pre, vload(&S.reg_limit)), min(wl, r0 + (long long)__builtin_popcountll(fm)));
    const int gp = vload(&S.global_pending);
    if (r0 >= lim || gp) {
      // stall attribution (cycles): 24 window full, 25 descriptor not prefetched, 26 global pending
      const unsigned long long n = mclk();
      PROF(if (lane == 0) S.prof[gp ? 26 : (r0 >= wl || !fm ? 24 : (r0 >= pre ? 25 : 27))] += n - t_poll);
      t_poll = n;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    lds_fence();
    const unsigned long long t0 = mclk();
    int nb = (int)min((long long)RB, lim - r0);
    // the batch's rows (prefetched by the previous iteration when it could)
    if (eb_first == r0 && eb_n > 0) nb = min(nb, eb_n);
    else fetch(r0, nb);
#if DGP_REG_PROBES
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the batch rows are in
    PROF(if (lane == 0) S.prof[16] += mclk() - t0);
#endif
    // the batch's slots: the lowest free ones (nb <= popcount(fm) by lim); lane b takes sb[b]
    int sb[RB];
    int my_s = 0;
    {
      SMask f = fm;
#pragma unroll
      for (int b = 0; b < RB; b++) {
        sb[b] = f ? __builtin_ctzll(f) : 0;
        if (lane == b) my_s = sb[b];
        if (b < nb) f &= f - 1;
      }
    }
    // ---------------------------------------------------------------- phase A
    // lane b: stimulus r0 + b. Flags (PRE's, plus the queue rule and debug modes), then the
    // batch ends after its first global stimulus (nothing registers behind a global)
    const long long ql = vload(&S.qlen);  // only globals grow the queue; none runs now
    const bool qglob = ql > 0 && (!S.inv_ok || !S.q_anon);
    const uint32_t fadd = (qglob ? F_GLOBAL : 0u) | ((D.dbg & 1) ? F_EXACT : 0u) | ((D.dbg & 2) ? F_GLOBAL : 0u);
    uint32_t fl = lane < nb ? (HB.x | fadd) : 0u;
    int nt = lane < nb ? (int)HB.y : 0;
    PROF(if (lane < nb && qglob && !(HB.x & F_GLOBAL)) atomicAdd(&S.prof[23], 1ull));  // diagnostics
    if (ballot(lane < nb && (fl & F_BADTOUCH))) {
      serr(S, SERR_RANGE, (int)r0);
      break;
    }
    const unsigned long long gm = ballot(lane < nb && (fl & F_GLOBAL));
    const bool glob_end = gm != 0;
    const int nbat = glob_end ? __builtin_ctzll(gm) + 1 : nb;
    const int nloc = nbat - (glob_end ? 1 : 0);  // stimuli with touch lists
    if (glob_end && lane == nbat - 1) fl |= F_TOUCHALL;
    if (lane >= nloc) nt = 0;
    {  // run continuations: this and the stimulus before it are F_SIMPLE on the same worker
      int w0 = -1;
#pragma unroll
      for (int b = 0; b < RB; b++) {
        const int v = b < nloc ? (rl(TB[b], 0) & T_W) : -1;
        if (lane == b) w0 = v;
      }
      const bool sim = lane < nloc && (fl & F_SIMPLE);
      int pw = __shfl_up(sim ? w0 : -1, 1);
      if (lane == 0) pw = prev_simple_w;
      if (sim && pw == w0) fl |= F_RUNM;
      prev_simple_w = rl(sim ? w0 : -1, nbat - 1);
    }
    if (lane < nbat) {
      L.ntouch[my_s] = nt;
      L.flags[my_s] = fl;
      L.pred[my_s] = BIG;
      L.predc[my_s] = 0;
      L.sid[my_s] = r0 + lane;
    }
    int ntb[RB];
#pragma unroll
    for (int b = 0; b < RB; b++) {  // the distinct touched workers (deduplicated by PRE), one lane each
      ntb[b] = b < nloc ? rl(nt, b) : 0;
      if (lane < ntb[b]) L.touch[sb[b]][lane] = (uint16_t)TB[b];
    }
    const unsigned long long tA = mclk();
    // ---------------------------------------------------------------- phase B
    lds_fence();  // the slots' LDS state is written before any mask bit can expose it
    if (lane == 0) {
      SMask taken = 0;
#pragma unroll
      for (int b = 0; b < RB; b++)
        if (b < nbat) taken |= 1ull << sb[b];
      atomicAnd(&S.freem, ~taken);
      vstore(&S.reg_pos, r0 + nbat);
      if (glob_end) vstore(&S.global_pending, 1);  // a global ends its batch
    }
    // every mask registration back to back (one wave's LDS atomics run in order)
    SMask oldb[RB];
#pragma unroll
    for (int b = 0; b < RB; b++) {  // every lane issues: an inactive lane ORs 0 into its own word
      oldb[b] = 0;
      if (b >= nloc) break;
      const bool on = lane < ntb[b];
      // entry 0 is the completing worker; a later entry flagged T_CAND is a frontier candidate
      // (candidate-only: the stimulus waits for it in place, before its frontier)
      const bool co = WAITC && lane > 0 && (TB[b] & T_CAND);
      const SMask bit = co ? slot_bits(sb[b]) : (1ull << sb[b]);
      oldb[b] = __hip_atomic_fetch_or(&P.mask[on ? (TB[b] & T_W) : lane], on ? bit : 0ull, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
    }
#if DGP_REG_PROBES
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the mask atomics returned
    const unsigned long long tM = mclk();
    PROF(if (lane == 0) S.prof[20] += tM - tA);
#endif
    // predecessor count of stimulus b = its workers that an earlier in-flight stimulus holds:
    // it waits on each for the latest one only, whose release of that worker wakes it
    // (release_worker picks the earliest successor). With wait-in-place claims each lane adds
    // its own count to the slot (pred, or predc for a candidate-only worker: no-return LDS
    // adds, in order after the guard); without them (the 64-slot build, registrar-bound on
    // C3) the count is summed per slot in registers, a ballot each, and added by the guard
    // drop below in the same atomic (same-box A/B, profiles/r06/registrar_fused_count_ab.txt:
    // C3 +0.5 %, C2 -0.6 % in the 32-slot build, which keeps the adds)
    int pc_my = 0;  // lane b: slot b's predecessor count (64-slot build)
#pragma unroll
    for (int b = 0; b < RB; b++) {
      if (b >= nloc) break;
      const int c = (lane < ntb[b] && (oldb[b] & ~(1ull << sb[b])) != 0) ? 1 : 0;
      if (WAITC) {
        const bool co = lane > 0 && (TB[b] & T_CAND);
        if (c) __hip_atomic_fetch_add(co ? &L.predc[sb[b]] : &L.pred[sb[b]], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        const int pb = __builtin_popcountll(ballot(c != 0));
        if (lane == b) pc_my = pb;
      }
    }
    if (glob_end) {  // a global stimulus waits for every in-flight stimulus on every worker
      const int sg = sb[nbat - 1];
      const SMask bit = 1ull << sg;
      int cnt = 0;
      for (int c = lane; c < D.W; c += 64)
        cnt += (__hip_atomic_fetch_or(&P.mask[c], bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & ~bit) != 0 ? 1 : 0;
      if (cnt) __hip_atomic_fetch_add(&L.pred[sg], cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
#if DGP_REG_PROBES
    PROF(if (lane == 0) S.prof[21] += mclk() - tM);
#endif
    // lane b drops slot b's registration guard; the count left is its predecessors not yet
    // released (releases that came first were never counted)
    if (lane < nbat) {
      const int op = __hip_atomic_fetch_add(&L.pred[my_s], pc_my - BIG, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (op + pc_my == BIG) atomicOr(&S.ready, 1ull << my_s);
      if (DGP_TRACE) {
        if (TRL) TR(r0 + lane, 0);
        if (TRL && op == BIG) TR(r0 + lane, 1);
        trace_at(D, r0 + lane, 7, (unsigned long long)((op + pc_my - BIG) | (nt << 16)));
      }
    }
    const unsigned long long tB = mclk();
    {  // prefetch the next batch's rows while the executors run
      const long long r1 = r0 + nbat;
      const int n1 = (int)min((long long)RB, pre - r1);
      if (n1 > 0) fetch(r1, n1);
      else eb_first = -1;
    }
    if (lane == 0) {
      t_poll = mclk();
      if (D.resident) S.t_role[2] = rclk();
      PROF(S.prof[3] += t_poll - t0);
      PROF(S.prof[31] += nbat);
      PROF(S.prof[27] += 1);            // batches
#if !DGP_PHASE_PROBES  // (probe builds use 16..23 for the executor phases)
      PROF(S.prof[17] += tA - t0);      // fetch wait + phase A
      PROF(S.prof[18] += tB - tA);      // phase B
      PROF(S.prof[19] += t_poll - tB);  // prefetch issue
#endif
    }
    lds_fence();
  }
}

// ===================================================================== executors
// needs_what of one worker (:800-823): LDS line in lanes 0..NLW-2, control word in lane
// NLW-1 (count of entries << 8 | 1 when overflow entries are in use; NL_OVF: scan mode),
// overflow entries in D.gw_needs_ext (global), scan mode = exact needed_elsewhere checks.
__device__ __forceinline__ bool st_needed_elsewhere(const Dev& D, int d, int w, int except) {
  for (int64_t k = D.dpt_ptr[d]; k < D.dpt_ptr[d + 1]; k++) {
    const int x = D.dpt_idx[k];
    if (x != except && D.proc_on[x] == w) return true;
  }
  return false;
}

// The bytes of deps [k0, k1) of task `except` (on worker c) that no other task on c
// needs: in scan mode needs_inc / needs_dec return exactly these, and change nothing,
// so the deps are taken 64 at a time (int64 sum: exact in any order).
__device__ __forceinline__ int64_t scan_needs_sum(const Dev& D, int64_t k0, int64_t k1, int c, int except) {
  int64_t v = 0;
  for (int64_t q = k0 + lane_id(); q < k1; q += 64) {
    const int d = D.dep_idx[q];
    if (holds_any(D, d, c)) continue;
    if (!st_needed_elsewhere(D, d, c, except)) v += nbv(D, D.res_nbytes[d]);
  }
  return wsum64(v);
}

template <bool LW>
__device__ __forceinline__ uint32_t line_load(const WPtr<LW>& P, int c) {
  return lane_id() < NLW ? P.needs[(size_t)c * NLW + lane_id()] : 0u;
}
template <bool LW>
__device__ __forceinline__ void line_store(const WPtr<LW>& P, int c, uint32_t nl) {
  if (lane_id() < NLW) P.needs[(size_t)c * NLW + lane_id()] = nl;
}
__device__ __forceinline__ int line_used(uint32_t nl) { return __builtin_popcountll(ballot(lane_id() < NLW - 1 && nl != 0)); }

// _dec_needs_replica for dependency d (held elsewhere) of the task leaving worker c
// (returns the bytes c no longer needs)
__device__ __attribute__((always_inline)) int64_t needs_dec(const Dev& D, SCtl& S, int c, uint32_t& nl, int d, int64_t nb, int except) {
  const int lane = lane_id();
  const uint32_t ctl = rlu(nl, NLW - 1);
  if (ctl == NL_OVF) return st_needed_elsewhere(D, d, c, except) ? 0 : nb;
  const unsigned long long m = ballot(lane < NLW - 1 && nl != 0 && (nl >> 8) == (uint32_t)d);
  if (m) {
    const int ml = __builtin_ctzll(m);
    const uint32_t v = rlu(nl, ml) - 1;
    const bool gone = (v & 0xffu) == 0;
    if (lane == ml) nl = gone ? 0u : v;
    if (gone && lane == NLW - 1) nl -= 0x100u;
    return gone ? nb : 0;
  }
  const int ext = (int)(ctl >> 8) - line_used(nl);
  if (ext > 0) {
    uint32_t* X = D.gw_needs_ext + (size_t)c * NXW;
    const uint32_t xe = lane < NXW ? __hip_atomic_load(X + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const unsigned long long mx = ballot(lane < NXW && xe != 0 && (xe >> 8) == (uint32_t)d);
    if (mx) {
      const int ml = __builtin_ctzll(mx);
      const uint32_t v = rlu(xe, ml) - 1;
      const bool gone = (v & 0xffu) == 0;
      if (lane == ml) __hip_atomic_store(X + ml, gone ? 0u : v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (gone && lane == NLW - 1) nl -= 0x100u;
      __threadfence_block();
      return gone ? nb : 0;
    }
  }
  // remove_from_processing decrements only what is in needs_what (:767-769): after replica
  // events (add_replica deletes the entry, :831-834) an entry may be gone
  if (D.evf & EVF_MULTI) return 0;
  serr(S, SERR_NEEDS, d);
  return 0;
}

// _inc_needs_replica for dependency d (not held by c) of task `except` placed on c
// (returns the bytes c newly needs)
__device__ __attribute__((always_inline)) int64_t needs_inc(const Dev& D, SCtl& S, int c, uint32_t& nl, int d, int64_t nb, int except) {
  const int lane = lane_id();
  const uint32_t ctl = rlu(nl, NLW - 1);
  if (ctl == NL_OVF) return st_needed_elsewhere(D, d, c, except) ? 0 : nb;
  const unsigned long long m = ballot(lane < NLW - 1 && nl != 0 && (nl >> 8) == (uint32_t)d);
  if (m) {
    const int ml = __builtin_ctzll(m);
    if ((rlu(nl, ml) & 0xffu) == 0xffu) {
      serr(S, SERR_NEEDS, d);
      return 0;
    }
    if (lane == ml) nl += 1;
    return 0;
  }
  const int used = line_used(nl);
  const int ext = (int)(ctl >> 8) - used;
  uint32_t* X = D.gw_needs_ext + (size_t)c * NXW;
  uint32_t xe = 0;
  if (ext > 0) {
    xe = lane < NXW ? __hip_atomic_load(X + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const unsigned long long mx = ballot(lane < NXW && xe != 0 && (xe >> 8) == (uint32_t)d);
    if (mx) {
      const int ml = __builtin_ctzll(mx);
      if ((rlu(xe, ml) & 0xffu) == 0xffu) {
        serr(S, SERR_NEEDS, d);
        return 0;
      }
      if (lane == ml) __hip_atomic_store(X + ml, xe + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_block();
      return 0;
    }
  }
  const unsigned long long em = ballot(lane < NLW - 1 && nl == 0);
  if (em) {
    if (lane == __builtin_ctzll(em)) nl = ((uint32_t)d << 8) | 1u;
    if (lane == NLW - 1) nl += 0x100u;
    return nb;
  }
  if (ext < NXW) {
    const unsigned long long ex = ballot(lane < NXW && xe == 0);
    const int ml = __builtin_ctzll(ex);
    if (lane == ml) __hip_atomic_store(X + ml, ((uint32_t)d << 8) | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == NLW - 1) nl = nl + 0x100u;
    __threadfence_block();
    return nb;
  }
  // full: scan mode from here on (only reached when every earlier stimulus has retired)
  if (lane == NLW - 1) nl = NL_OVF;
  return nb;
}

// All of one task's dependency entries at once. A task's dependencies are distinct, so
// their needs_what entries are distinct lanes of the line: each dependency is matched
// against the line in one compare (no readlane chain through the line). Fast path only
// when every entry of c lives in the LDS line (no overflow entries, not scan mode) and
// the outcome needs no overflow entry; otherwise false with nl untouched, and the caller
// takes the one-at-a-time path (needs_dec / needs_inc).
// _dec_needs_replica (:815-823) for the dependencies in entries L0.. of E not held by c;
// freed = the bytes c no longer needs.
// lane masks of a comparison over the (active) lanes: one v_cmp into an SGPR pair
__device__ __forceinline__ unsigned long long lm_eq(unsigned a, unsigned b) { return __builtin_amdgcn_uicmp(a, b, 32); }
__device__ __forceinline__ unsigned long long lm_ne(unsigned a, unsigned b) { return __builtin_amdgcn_uicmp(a, b, 33); }
__device__ __forceinline__ bool lm_has(unsigned long long m) { return (m >> lane_id()) & 1ull; }
constexpr unsigned long long NL_LINE = (1ull << (NLW - 1)) - 1;  // the line's entry lanes

__device__ __forceinline__ bool needs_dec_all(const uint4& E, int L0, int k, int c, uint32_t& nl, int64_t& freed) {
  const uint32_t ctl = rlu(nl, NLW - 1);
  const unsigned long long used = lm_ne(nl, 0u) & NL_LINE;
  if (ctl == NL_OVF || (int)(ctl >> 8) != __builtin_popcountll(used)) return false;
  const uint32_t key = nl >> 8;
  const unsigned long long one = lm_eq(nl & 0xffu, 1u) & used;  // entries this decrement empties
  unsigned long long hit = 0;
  int64_t fr = 0;
  int ngone = 0;
  for (int i = 0; i < k; i++) {
    if (rl((int)E.y, L0 + i) == c) continue;  // held by c: never needed
    const unsigned long long m = lm_eq(key, rlu(E.x, L0 + i)) & used;
    if (!m) return false;  // not in the line (overflow / replica events): the general path
    hit |= m;
    if (m & one) {
      fr += mk64(rlu(E.z, L0 + i), rlu(E.w, L0 + i));
      ngone++;
    }
  }
  if (hit) nl = lm_has(hit & one) ? 0u : (lm_has(hit) ? nl - 1u : nl);
  if (ngone) nl = lane_id() == NLW - 1 ? nl - ((uint32_t)ngone << 8) : nl;
  freed = fr;
  return true;
}

// _inc_needs_replica (:800-813) for the dependencies in entries L0.. of E not held by c
// (task placed on c); added = the bytes c newly needs.
__device__ __forceinline__ bool needs_inc_all(const uint4& E, int L0, int k, int c, uint32_t& nl, int64_t& added) {
  const uint32_t ctl = rlu(nl, NLW - 1);
  const unsigned long long used = lm_ne(nl, 0u) & NL_LINE;
  if (ctl == NL_OVF || (int)(ctl >> 8) != __builtin_popcountll(used)) return false;
  const uint32_t key = nl >> 8;
  const unsigned long long full = lm_eq(nl & 0xffu, 0xffu) & used;
  unsigned long long freem = ~used & NL_LINE;
  unsigned long long hit = 0;
  uint32_t nn = nl;
  int64_t ad = 0;
  int nins = 0;
  for (int i = 0; i < k; i++) {
    if (rl((int)E.y, L0 + i) == c) continue;
    const uint32_t d = rlu(E.x, L0 + i);
    const unsigned long long m = lm_eq(key, d) & used;  // against the line as loaded (deps are distinct)
    if (m) {
      if (m & full) return false;
      hit |= m;
    } else {
      if (!freem) return false;  // the line is full: the general path (overflow entries)
      const int l = __builtin_ctzll(freem);
      freem &= freem - 1;
      nn = lane_id() == l ? (d << 8) | 1u : nn;
      ad += mk64(rlu(E.z, L0 + i), rlu(E.w, L0 + i));
      nins++;
    }
  }
  if (hit) nn = lm_has(hit) ? nn + 1u : nn;
  if (nins) nn = lane_id() == NLW - 1 ? nn + ((uint32_t)nins << 8) : nn;
  nl = nn;
  added = ad;
  return true;
}

// a worker with nothing processing needs nothing (leave scan / overflow mode)
__device__ __attribute__((always_inline)) void needs_reset(const Dev& D, int c, uint32_t& nl) {
  const int lane = lane_id();
  const uint32_t ctl = rlu(nl, NLW - 1);
  if (ctl == NL_OVF || (ctl >> 8) != 0) {
    if (lane < NXW) __hip_atomic_store(D.gw_needs_ext + (size_t)c * NXW + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence_block();
  }
  if (lane < NLW) nl = 0;
}

// per-stimulus outputs, staged as they are made: the values are wave-uniform, lane 0
// stores each record / placement into the slot's staging rows at once (nothing is held in
// registers until the slot retires)
struct Out {
  int nrec, npl;
  size_t st0;  // the slot's staging base (slot * PLC)
  __device__ void rec(const Dev& D, int kind, int w, int p, int64_t dnet, double occ, int np, int task, double dur) {
    if (lane_id() == 0 && nrec < PLC) {
      SRec rc;
      rc.w = w;
      rc.p = (int16_t)p;
      rc.kind = (int8_t)kind;
      rc.pad = 0;
      rc.nproc = np;
      rc.task = task;
      rc.dnet = dnet;
      rc.occ = occ;
      rc.dur = dur;
      D.srec[st0 + nrec] = rc;
    }
    nrec++;
  }
  __device__ void place(const Dev& D, int task, int w, int64_t comm, double start, int64_t wsnb, int route) {
    if (lane_id() == 0 && npl < PLC) {
      D.s2_task[st0 + npl] = task;
      D.s2_worker[st0 + npl] = w;
      D.s2_comm[st0 + npl] = comm;
      D.s2_start[st0 + npl] = start;
      D.s2_wsnb[st0 + npl] = wsnb;
      D.s2_route[st0 + npl] = (int8_t)route;
    }
    npl++;
  }
};

// WorkerState.add_to_processing / remove_from_processing on the dict of c (:733-771)
template <bool LW>
__device__ __forceinline__ bool dict_update(const WPtr<LW>& P, int c, int p, int delta, WDict& d) {
  using U4 = typename WPtr<LW>::template P<Q4>;
  d = dict_load<LW>(P, c);
  const bool ok = dict_add(d, p, delta);
  if (lane_id() == 0) {
    st4(ascast<U4>(P.pcnt + (size_t)c * PD), d.c);
    st4(ascast<U4>(P.pcnt + (size_t)c * PD + 4), d.c1);
    P.plen[c] = d.ord;
  }
  return ok;
}

// release worker c of slot s: clear the slot's bit. Every bit left on c belongs to a later
// stimulus (an earlier one holding c would have released it before s could run); the earliest
// of them is the one waiting for s on c, and it alone counted s (role_reg): it counts down.
// With WAITC the high half of the old mask says, per successor, whether it registered the
// worker as a candidate only: its candidate count (predc) counts down instead.
__device__ __forceinline__ int release_succ(SLds& L, SMask old, int from = -1) {  // -> the slot made ready, or -1
  const SMask succ = WAITC ? (old & 0xffffffffull) : old;
  if (!succ) return -1;
  int bs = __builtin_ctzll(succ);
  long long best = vload(&L.sid[bs]);
  for (SMask m = succ & (succ - 1); m; m &= m - 1) {
    const int b = __builtin_ctzll(m);
    const long long v = vload(&L.sid[b]);
    if (v < best) {
      best = v;
      bs = b;
    }
  }
  if (WAITC && ((old >> 32) >> bs) & 1ull) {
    const int pc = __hip_atomic_fetch_add(&L.predc[bs], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (TR3 && pc == 1) {
      const Dev& D = c_dev;
      TR(L.sid[bs], 20);
      if (from >= 0) trace_at(D, L.sid[bs], 21, (unsigned long long)L.sid[from]);
    }
    return -1;
  }
  if (atomicSub(&L.pred[bs], 1) == 1) {
    atomicOr(&L.c.ready, 1ull << bs);
    if (TRL) {
      const Dev& D = c_dev;
      TR(L.sid[bs], 1);
      if (TR3 && from >= 0) trace_at(D, L.sid[bs], 19, (unsigned long long)L.sid[from]);
    }
    return bs;
  }
  return -1;
}
template <bool LW>
__device__ __forceinline__ int release_worker(SLds& L, const WPtr<LW>& P, int s, int c) {
  const SMask bit = slot_bits(s);
  return release_succ(L, __hip_atomic_fetch_and(&P.mask[c], ~bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & ~bit,
                      DGP_TRACE ? s : -1);
}

// release the workers of slot s (the waiting successors may run) — LDS state only
template <bool LW>
__device__ __attribute__((always_inline)) void release_slot(const Dev& D, SLds& L, const WPtr<LW>& P, int s, bool all) {
  const int lane = lane_id();
  const SMask bit = slot_bits(s);
  auto rel = [&](int c) {
    release_succ(L, __hip_atomic_fetch_and(&P.mask[c], ~bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & ~bit,
                 DGP_TRACE ? s : -1);
  };
  if (all) {
    for (int c = lane; c < D.W; c += 64) rel(c);
  } else {
    const int nt = L.ntouch[s];
    if (lane < nt) rel((int)L.touch[s][lane] & T_W);
  }
}

// publish the counts in the retire ring, mark the stimulus done and free its slot: the
// sequencer retires it in order later (its staging rows were written as the outputs were made)
template <class O>
__device__ __attribute__((always_inline)) void finish_slot(const Dev& D, SLds& L, int s, long long r, const O& o, int npops, bool direct) {
  const int lane = lane_id();
  const int q = (int)(r & (RS - 1));
  if (lane == 0) {
    RMeta me;
    me.npl = o.npl;
    me.nrec = (uint8_t)(direct ? 0 : o.nrec);
    me.npops = (uint8_t)npops;
    me.direct = direct ? 1 : 0;
    me.pad = 0;
    L.rmeta[q] = me;
  }
  __threadfence_block();
  if (lane == 0) {
    vstore(&L.rdone[q], r + 1);
    atomicOr(&L.c.freem, 1ull << s);  // the slot may take the next registration
  }
  if (DGP_TRACE && lane == 0) TR(r, 5);
}

// wave minimum (uniform): DPP within rows of 16 lanes (quad swaps, half-row and row
// mirrors), then the four row results
__device__ __forceinline__ unsigned wmin_u32(unsigned v) {
  v = min(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xb1, 0xf, 0xf, false));   // quad_perm(1,0,3,2)
  v = min(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4e, 0xf, 0xf, false));   // quad_perm(2,3,0,1)
  v = min(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = min(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xf, 0xf, false));  // row_mirror
  return min(min(rlu(v, 0), rlu(v, 16)), min(rlu(v, 32), rlu(v, 48)));
}

// objective key of lane's candidate: worker_objective (:3131-3146) + canonical index
struct Key {
  double start;
  int64_t nb;
  int w;
  int64_t comm;
};
__device__ __forceinline__ bool key_less(const Key& a, const Key& b) {
  if (a.start != b.start) return a.start < b.start;
  if (a.nb != b.nb) return a.nb < b.nb;
  return a.w < b.w;
}
__device__ __forceinline__ Key key_at(const Key& k, int l) {
  Key o;
  o.start = mkd(rlu(dlo(k.start), l), rlu(dhi(k.start), l));
  o.nb = mk64(rlu(lo32(k.nb), l), rlu(hi32(k.nb), l));
  o.w = rl(k.w, l);
  o.comm = mk64(rlu(lo32(k.comm), l), rlu(hi32(k.comm), l));
  return o;
}

// start time as a u64 whose unsigned order is key_less's fp64 order (+0 and -0 equal)
__device__ __forceinline__ uint64_t start_key(double x) {
  const uint64_t b = x == 0.0 ? 0ull : (uint64_t)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  return ((uint64_t)rlu((unsigned)(v >> 32), l) << 32) | rlu((unsigned)v, l);
}

// the resolved durations of a stimulus (descriptor entries 3..6, in lanes 3..6 of E) into
// the executor wave's LDS table, read by prefix id (one wave's LDS operations run in order)
__device__ __forceinline__ DTab stim_durations(const Dev& D, SLds& L, const uint4& E, long long r) {
  const int lane = lane_id();
  const auto t = (__attribute__((address_space(3))) double*)(double*)L.dur[threadIdx.x >> 6];
  if (D.P <= PD) {
    if (lane >= 3 && lane < 7) {
      t[2 * (lane - 3)] = mkd(E.x, E.y);
      t[2 * (lane - 3) + 1] = mkd(E.z, E.w);
    }
  } else if (lane < D.P) {  // more prefixes than the descriptor carries: the stimulus' row
    t[lane] = D.dring[(size_t)(r & (DR - 1)) * PX + lane];
  }
  return (DTab)(const double*)t;
}

// a stimulus whose effects stay on the workers it registered. Returns false (nothing
// changed) when it needs every earlier stimulus retired first (needs scan mode).
template <bool LW>
__device__ __attribute__((always_inline)) bool exe_local(const Dev& D, SLds& L, const WPtr<LW>& P, int s, long long r, int qmode, bool exact, const uint4& E,
                                                         int& woke) {
  // WAITC: the candidate-only workers (touch entries > 0 flagged T_CAND) may still be held by
  // earlier stimuli when this one starts; their state is read after the wait before the frontier
  SCtl& S = L.c;
  const int lane = lane_id();
  const DTab durv = stim_durations(D, L, E, r);
  const int t = rl((int)E.x, 0), w = rl((int)E.y, 0), p = rl((int)E.z, 0);
  const uint32_t flags = rlu(E.w, 0);
  const int64_t nbt = mk64(rlu(E.x, 1), rlu(E.y, 1));
  const unsigned cnts = rlu(E.z, 1);
  const int kt = cnts & 0xff, nrel = (cnts >> 8) & 0xff, nf = (cnts >> 16) & 0xff;
  const double dobs = mkd(rlu(E.x, 2), rlu(E.y, 2));
  const int TD = E_HDR, RL0 = E_HDR + kt, FX0 = RL0 + nrel;
#if DGP_PHASE_PROBES
  unsigned long long tph = mclk();
  auto phase = [&](int k) {
    const unsigned long long n = mclk();
    PROF(if (lane == 0) atomicAdd(&S.prof[k], n - tph));
    tph = n;
  };
#else
  auto phase = [](int) {};
#endif
  // ---- capacity check of the needs tables this stimulus may grow
  const int tot_new = rl((int)E.w, 2);  // the frontier's dependency count (prefetcher)
  if (!exact) {
    const int ntch = L.ntouch[s];
    bool bad = false;
    if (lane < ntch) {
      const int tv0 = L.touch[s][lane];
      const int c = tv0 & T_W;
      const uint32_t ctl = P.needs[(size_t)c * NLW + NLW - 1];
      // a candidate-only worker's table may still grow by earlier stimuli's commits: margin
      const int slack = (WAITC && lane > 0 && (tv0 & T_CAND)) ? NXW / 2 : 0;
      bad = ctl == NL_OVF || (int)(ctl >> 8) + tot_new + slack > NLW - 1 + NXW;
    }
    if (ballot(bad)) return false;
  }
  Out o;
  o.nrec = 0;
  o.npl = 0;
  o.st0 = (size_t)(r & (RS - 1)) * PLC;
  phase(11);
  if (DGP_TRACE == 2 && lane == 0) TR(r, 0);
  if (TR3 && lane == 0) TR(r, 8);
  // ---- the touched workers' state, one lane each, in registers for the whole stimulus
  const int nt = L.ntouch[s];
  const bool tl = lane < nt;
  const int tv = tl ? (int)L.touch[s][lane] : 0;
  const int cj = tv & T_W;
  const bool candl = (tv & T_CAND) != 0;  // a holder of a frontier task's dependency
  const bool wc = WAITC && tl && lane > 0 && candl;  // candidate-only: read after the wait
  int np = 0, nth = 1;
  WDict dj;
  dj.c = make_uint4(0, 0, 0, 0);
  dj.c1 = make_uint4(0, 0, 0, 0);
  dj.ord = 0;
  int64_t net = 0, nbj = 0;
  if (tl) nth = P.nthreads[cj];  // static while stimuli run
  if (tl && !wc) {
    np = P.nproc[cj];
    dj = dict_load<LW>(P, cj);
    net = P.netocc[cj];
    nbj = P.nbytes[cj];
  }
  const int capw = P.cap[w];
  uint32_t nl = line_load<LW>(P, w);
  const unsigned long long wm = ballot(tl && cj == w);
  if (!wm) {
    serr(S, SERR_INV, 700000000 + (int)r);
    return true;
  }
  const int jw = __builtin_ctzll(wm);
  const bool isw = lane == jw;
  double nbw = net_bw_of(net, D);            // this lane's netocc / bandwidth
  const bool nth1 = !ballot(tl && nth != 1);  // occ / 1.0 == occ: the division is skipped
  phase(16);
  if (DGP_TRACE == 2 && lane == 0) TR(r, 1);
  if (TR3 && lane == 0) {
    TR(r, 9);
    trace_at(D, r, 22, (unsigned long long)(nf | kt << 8 | nrel << 16 | nt << 24));
    trace_at(D, r, 23, (unsigned long long)vload(&L.predc[s]));
  }
  // ------------------------------------------- completion: processing -> memory (:2366)
  int64_t dnet = 0;
  int64_t freed = 0;
  if (needs_dec_all(E, TD, kt, w, nl, freed)) dnet = -freed;
  else for (int i = 0; i < kt; i++) {  // _dec_needs_replica for the dependencies w needed
    const int L_ = TD + i;
    const int h = rl((int)E.y, L_);
    if (h == w) continue;
    const int d = rl((int)E.x, L_);
    const int64_t nb = mk64(rlu(E.z, L_), rlu(E.w, L_));
    dnet -= needs_dec(D, S, w, nl, d, nb, t);
  }
  const int npw = rl(np, jw) - 1;
  if (npw == 0) needs_reset(D, w, nl);
  line_store<LW>(P, w, nl);
  if (isw) {
    dict_add(dj, p, -1);
    np = npw;
    net += dnet;
  }
  if (dnet != 0) nbw = net_bw_of(net, D);  // dnet is uniform
  phase(17);
  if (DGP_TRACE == 2 && lane == 0) TR(r, 3);
  if (TR3 && lane == 0) TR(r, 10);
  // every lane's occupancy and stack time, kept current: only w (now) and each chosen
  // worker (after its commit) change during the stimulus
  double occj = occ_dict_r(dj, nbw, durv, D);
  double stkj = nth1 ? occj : occj / (double)nth;
  o.rec(D, K_COMPLETE, w, p, dnet, mkd(rlu(dlo(occj), jw), rlu(dhi(occj), jw)), npw, t, dobs);
  // add_replica (:3148), then the releases popped before the frontier (LIFO, :3309-3314)
  if (isw) nbj += (flags & F_SELFREL) ? 0 : nbt;
  for (int i = 0; i < nrel; i++) {
    const int h = rl((int)E.x, RL0 + i);
    const int64_t nb = mk64(rlu(E.z, RL0 + i), rlu(E.w, RL0 + i));
    if (tl && !wc && cj == h) nbj -= nb;
  }
  // a release-only holder (ws.nbytes of a released dependency; no frontier candidate) is final
  // now: written back and released before the frontier
  bool released = false;  // this lane's worker was written back and released early
  {
    const bool ro = tl && !isw && !candl;
    if (ballot(ro)) {
      if (ro) P.nbytes[cj] = nbj;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the state above is in LDS
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      if (ro) release_worker<LW>(L, P, s, cj);
      released = ro;
    }
  }
  if (TR3 && lane == 0) TR(r, 11);
  if (WAITC && ballot(wc)) {
    // ---- the candidates: every earlier stimulus holding one has released it (release_succ
    // counts predc down), then their state, with this stimulus' releases applied
    if (vload(&L.predc[s]) != 0) {
      if (DGP_EXE_PRIO) __builtin_amdgcn_s_setprio(1);
      while (vload(&L.predc[s]) != 0) __builtin_amdgcn_s_sleep(1);
      if (DGP_EXE_PRIO) __builtin_amdgcn_s_setprio(3);
    }
    lds_fence();
    if (wc) {
      np = P.nproc[cj];
      dj = dict_load<LW>(P, cj);
      net = P.netocc[cj];
      nbj = P.nbytes[cj];
    }
    for (int i = 0; i < nrel; i++) {
      const int h = rl((int)E.x, RL0 + i);
      const int64_t nb = mk64(rlu(E.z, RL0 + i), rlu(E.w, RL0 + i));
      if (wc && cj == h) nbj -= nb;
    }
    if (wc) {
      nbw = net_bw_of(net, D);
      occj = occ_dict_r(dj, nbw, durv, D);
      stkj = nth1 ? occj : occj / (double)nth;
    }
    if (!exact) {  // the candidates' needs tables, exactly now (the claim checked them with a margin)
      bool bad = false;
      if (wc) {
        const uint32_t ctl = P.needs[(size_t)cj * NLW + NLW - 1];
        bad = ctl == NL_OVF || (int)(ctl >> 8) + tot_new > NLW - 1 + NXW;
      }
      if (ballot(bad)) {  // rare: continue as the oldest stimulus (every earlier one retired)
        while (vload(&S.seq_pos) != r) __builtin_amdgcn_s_sleep(1);
        lds_fence();
        exact = true;
      }
    }
  }
  phase(12);
  if (DGP_TRACE == 2 && lane == 0) TR(r, 4);
  if (TR3 && lane == 0) TR(r, 12);
  // ------------------------------ frontier in ascending priority: decide_worker (:8550)
  int off = FX0;
  for (int j = 0; j < nf; j++) {
    const int x = rl((int)E.x, off), px = rl((int)E.y, off);
    const int hz = rl((int)E.z, off);
    const int kx = hz & 0xff, nc = (hz >> 8) & 0xff;  // nc: a restricted task's resolved candidates
    // candidates = the holders of x's dependencies (each a touched lane); comm_bytes (:3136)
    int64_t comm = 0;
    bool cand = false;
    for (int i = 0; i < kx; i++) {
      const int L2 = off + 1 + i;
      const int hi = rl((int)E.y, L2);
      const int64_t nbi = mk64(rlu(E.z, L2), rlu(E.w, L2));
      if (cj == hi) cand = true;
      else comm += nbi;
    }
    if (hz & (1 << 16)) {  // restricted: the candidates PRE resolved (:8575-8586)
      cand = false;
      for (int i = 0; i < nc; i++) cand = cand || cj == rl((int)E.x, off + 1 + kx + i);
    }
    cand = cand && tl;
    Key k;
    k.start = stkj + (double)comm / (double)D.bandwidth;
    k.nb = nbj;
    k.w = cj;
    k.comm = comm;
    phase(18);
    if (TR3 && lane == 0 && j == 0) TR(r, 13);
    const unsigned long long cm = ballot(cand);
    if (!cm) {
      serr(S, SERR_CAND, x);
      return true;
    }
    Key best = key_at(k, __builtin_ctzll(cm));
    int jb = __builtin_ctzll(cm);
    for (unsigned long long rm = cm & (cm - 1); rm; rm &= rm - 1) {
      const int jq = __builtin_ctzll(rm);
      const Key q = key_at(k, jq);
      if (key_less(q, best)) {
        best = q;
        jb = jq;
      }
    }
    const int cb = best.w;
    if (j == nf - 1 && nt > 2) {
      // the last frontier decision is made: every touched worker but w and the chosen one
      // is final now (the non-chosen candidates were only read, the release holders were
      // settled before the frontier). Write them back and release them before the commit,
      // so stimuli waiting only on them do not wait for it.
      const bool early = tl && !isw && lane != jb && !released;
      if (ballot(early)) {
        if (early) {
          using U4 = typename WPtr<LW>::template P<Q4>;
          P.nproc[cj] = np;
          st4(ascast<U4>(P.pcnt + (size_t)cj * PD), dj.c);
          st4(ascast<U4>(P.pcnt + (size_t)cj * PD + 4), dj.c1);
          P.plen[cj] = dj.ord;
          P.netocc[cj] = net;
          P.nbytes[cj] = nbj;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the state above is in LDS
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (early) release_worker<LW>(L, P, s, cj);
        released = released || early;
        if (TRL && lane == 0) TR(r, 3);
      }
    }
    phase(19);
    if (TR3 && lane == 0 && j == 0) TR(r, 14);
    // _add_to_processing (:3199): record, WorkerState.add_to_processing, check_idle_saturated
    o.place(D, x, cb, best.comm, best.start, best.nb, ROUTE_NONROOTISH);
    uint32_t nlc = line_load<LW>(P, cb);
    if (exact) {  // scan mode reads processing_on of this stimulus' earlier placements
      __threadfence_block();
    }
    int64_t dn = 0;
    if (!needs_inc_all(E, off + 1, kx, cb, nlc, dn)) for (int i = 0; i < kx; i++) {
      const int L2 = off + 1 + i;
      if (rl((int)E.y, L2) == cb) continue;
      const int d = rl((int)E.x, L2);
      const int64_t nb = mk64(rlu(E.z, L2), rlu(E.w, L2));
      dn += needs_inc(D, S, cb, nlc, d, nb, x);
    }
    line_store<LW>(P, cb, nlc);
    const bool isb = lane == jb;
    bool okp = true;
    if (isb) {
      okp = dict_add(dj, px, +1);
      np += 1;
      net += dn;
    }
    if (dn != 0) nbw = isb ? net_bw_of(net, D) : nbw;  // dn is uniform
    if (ballot(!okp)) serr(S, SERR_PREFIX, x);
    if (exact && lane == 0) {  // scan mode reads them for this stimulus' later decisions (the
      D.proc_on[x] = cb;       // sequencer writes them, and the group count, at retirement)
      D.state[x] = S_PROCESSING;
    }
    occj = occ_dict_r(dj, nbw, durv, D);
    stkj = nth1 ? occj : occj / (double)nth;
    o.rec(D, K_PLACE, cb, px, dn, mkd(rlu(dlo(occj), jb), rlu(dhi(occj), jb)), rl(np, jb), x, 0.0);
    off += 1 + kx + nc;
    phase(20);
    if (TR3 && lane == 0 && j == 0) TR(r, 15);
  }
  if (DGP_TRACE == 2 && lane == 0) TR(r, 6);
  if (TR3 && lane == 0) TR(r, 16);
  // ---- every touched worker but w is final: write back and release it now (its waiting
  // successors may run while w takes the queue refill)
  if (tl && !isw && !released) {
    using U4 = typename WPtr<LW>::template P<Q4>;
    P.nproc[cj] = np;
    st4(ascast<U4>(P.pcnt + (size_t)cj * PD), dj.c);
    st4(ascast<U4>(P.pcnt + (size_t)cj * PD + 4), dj.c1);
    P.plen[cj] = dj.ord;
    P.netocc[cj] = net;
    P.nbytes[cj] = nbj;
  }
  if (nt > 1) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (tl && !isw && !released) release_worker<LW>(L, P, s, cj);
  }
  if (TRL && lane == 0) TR(r, 4);
  // -------------- stimulus_queue_slots_maybe_opened (:4983): only w can have open slots
  int pops = 0;
  if (qmode != 0 && !D.sat_inf) {
    const int slots = capw - rl(np, jw);
    if (slots > capw || o.npl + slots > PLC - 1) {
      serr(S, SERR_INV, 600000000 + (int)r);
      return true;
    }
    if (slots > 0) {
      pops = slots;
      if (qmode == 3) pops = (int)min((long long)slots, vload(&S.qlen));
    }
    const int qp = S.q_prefix;
    for (int i = 0; i < pops; i++) {
      const double st = stkj + 0.0 / (double)D.bandwidth;
      o.place(D, -1, w, 0, mkd(rlu(dlo(st), jw), rlu(dhi(st), jw)), mk64(rlu(lo32(nbj), jw), rlu(hi32(nbj), jw)),
              ROUTE_ROOTISH_Q);
      bool okq = true;
      if (isw) {
        okq = dict_add(dj, qp, +1);
        np += 1;
      }
      if (ballot(!okq)) serr(S, SERR_PREFIX, -1);
      occj = occ_dict_r(dj, nbw, durv, D);
      stkj = nth1 ? occj : occj / (double)nth;
      o.rec(D, K_PLACE, w, qp, 0, mkd(rlu(dlo(occj), jw), rlu(dhi(occj), jw)), rl(np, jw), -1, 0.0);
    }
  }
  if (TR3 && lane == 0) TR(r, 17);
  // ---- w written back last, then released
  if (isw) {
    using U4 = typename WPtr<LW>::template P<Q4>;
    P.nproc[cj] = np;
    st4(ascast<U4>(P.pcnt + (size_t)cj * PD), dj.c);
    st4(ascast<U4>(P.pcnt + (size_t)cj * PD + 4), dj.c1);
    P.plen[cj] = dj.ord;
    P.netocc[cj] = net;
    P.nbytes[cj] = nbj;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the state above is in LDS
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  int wk = -1;
  if (lane == jw) wk = release_worker<LW>(L, P, s, w);
  if (TR3 && lane == 0) TR(r, 18);
  woke = rl(wk, jw);  // the stimulus next on w, if this release made it ready
  phase(13);
  // ------------------------------------------------ retire: LDS state, then successors
  phase(21);
  // the completed task's and the releases' TaskState fields in HBM are written by the
  // sequencer when it retires the slot (seq_bookkeeping): nothing reads them before
  phase(14);
  finish_slot(D, L, s, r, o, pops, false);
  phase(15);
  return true;
}

// ============================================================ single-worker runs
// A run of consecutive stimuli r, r+1, ..., r+k-1 that each touch only worker w, place
// nothing (empty frontier), whose dependency w holds or needs from elsewhere (then the same
// dependency d0 for every such member, whose needs_what entry on w stays >= 1: a count
// decrement, no network-occupancy change) and whose releases are on w, with the queue
// empty: each is the completion bookkeeping of one task
// on w (_transition_processing_memory :2366-2442 -> _exit_processing_common :3258-3281 ->
// WorkerState.remove_from_processing :759-771, add_replica :3148, the releases :3309-3314;
// stimulus_queue_slots_maybe_opened :4983 finds no queued task). Each waits only for the
// one before it on w, so one executor runs them back to back on w's state: one claim and
// one release of w for the whole run instead of one per stimulus (the P2P-shuffle unpack
// completions on the barrier's worker, C3). The same fp64 operations in the same order as
// exe_local. Returns false (nothing done) when stimulus r itself is not of that form.
template <bool LW>
__device__ __attribute__((always_inline)) bool exe_run(const Dev& D, SLds& L, const WPtr<LW>& P, int s, long long r,
                                                       const uint4& E) {
  SCtl& S = L.c;
  const int lane = lane_id();
  if (L.ntouch[s] != 1) return false;
  const int w = rl((int)E.y, 0);
  // members: registered slots (guard dropped) whose stimulus r + k touches only w and waits
  // only for its predecessor on w; lane k (k >= 1) gets the slot of r + k, k consecutive
  const bool sl = lane < WIN && lane != s;
  const long long offl = sl ? vload(&L.sid[lane]) - r : -1;
  const bool el = sl && offl >= 1 && offl < 64 && vload(&L.pred[lane]) == 1 && vload(&L.ntouch[lane]) == 1 &&
                  (L.touch[lane][0] & T_W) == w && (vload(&L.flags[lane]) & (F_GLOBAL | F_EXACT | F_SIMPLE)) == F_SIMPLE;
  int my_slot = lane == 0 ? s : -1;
  int n = 1;
  while (n < 64) {
    const unsigned long long m = ballot(el && offl == n);
    if (!m) break;
    if (lane == n) my_slot = __builtin_ctzll(m);
    n++;
  }
  // each candidate's descriptor header (lane i: stimulus r + i); the dependency and release
  // entries are read whether present or not (a row always holds NE entries)
  uint4 h0 = make_uint4(0, 0, 0, 0), h1 = h0, h2 = h0, ed = h0, er = h0, dq[4];
  bool ok = false, needs_m = false;
  if (lane < n) {
    const uint4* row = D.desc + (size_t)((r + lane) & (DR - 1)) * NE;
    h0 = row[0];
    h1 = row[1];
    h2 = row[2];
#pragma unroll
    for (int q = 0; q < 4; q++) dq[q] = row[3 + q];
    ed = row[E_HDR];
    er = row[E_HDR + 1];
  }
  {
    bool same = true;  // the resolved durations equal the head's (one table serves the run)
#pragma unroll
    for (int q = 0; q < 4; q++)
      same = same && dq[q].x == rlu(E.x, 3 + q) && dq[q].y == rlu(E.y, 3 + q) && dq[q].z == rlu(E.z, 3 + q) &&
             dq[q].w == rlu(E.w, 3 + q);
    const int kt = h1.z & 0xff, nrel = (h1.z >> 8) & 0xff, nf = (h1.z >> 16) & 0xff;
    const uint4 erel = kt == 0 ? ed : er;
    ok = lane < n && (int)h0.y == w && !(h0.w & F_GLOBAL) && nf == 0 && kt <= 1 && nrel <= 1 &&
         (nrel == 0 || (int)erel.x == w) && same;
    er = erel;
    needs_m = ok && kt == 1 && (int)ed.y != w;  // _dec_needs_replica (:767-769) of a dependency held elsewhere
  }
  // the members that need a dependency from elsewhere all need the same one, d0, whose entry
  // in w's LDS needs_what line keeps a count >= 1 through the run (no entry leaves, so
  // netocc and the occupancy's network term stay as they are)
  const unsigned long long nm = ballot(needs_m);
  const uint32_t nl = line_load<LW>(P, w);
  const uint32_t ctl = rlu(nl, NLW - 1);
  if (ctl == NL_OVF) return false;  // scan mode: exe_local
  unsigned long long cut = ballot(!ok);
  int d_ml = -1;  // the line lane of d0's entry
  if (nm) {
    const uint32_t d0 = rlu(ed.x, __builtin_ctzll(nm));
    cut |= ballot(needs_m && ed.x != d0);
    const unsigned long long em = ballot(lane < NLW - 1 && nl != 0 && (nl >> 8) == d0);
    if (!em) {
      cut |= nm & (0ull - nm);  // d0 not in the line: the run ends before its first member
    } else {
      d_ml = __builtin_ctzll(em);
      const int c0 = (int)(rlu(nl, d_ml) & 0xffu);
      // the member whose decrement would empty the entry ends the run (exe_local takes it)
      unsigned long long mm = nm;
      for (int i = 1; i < c0 && mm; i++) mm &= mm - 1;
      if (mm) cut |= mm & (0ull - mm);
    }
  }
  int k = (int)min((unsigned long long)n, (unsigned long long)__builtin_ctzll(cut | (1ull << 63)));
  // a needs line with entries belongs to tasks still processing on w: w keeps one (no
  // needs_reset), as it does when the line is empty only if nothing else is processing
  if (ctl != 0) k = min(k, P.nproc[w] - 1);
  if (k <= 0) return false;
  const int n_dec = __builtin_popcountll(nm & ((k >= 64 ? 0ull : (1ull << k)) - 1ull));
  // the members leave the window's wake-up protocol: the guard keeps them from becoming ready
  if (lane >= 1 && lane < k) {
    const int op = __hip_atomic_fetch_add(&L.pred[my_slot], BIG, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (op != 1) serr(S, SERR_INV, 800000000 + (int)r);
  }
  // w's state, uniform in every lane; netocc does not change in the run
  int np = P.nproc[w];
  WDict dj = dict_load<LW>(P, w);
  const int64_t net = P.netocc[w];
  int64_t nbj = P.nbytes[w];
  const double nbw = net_bw_of(net, D);
  const DTab durv = stim_durations(D, L, E, r);
  // members of one prefix whose count on w stays >= 1 (no dict entry leaves): member i's
  // state is the head's with i + 1 completions applied, so every member's occupancy and
  // record is made at once, lane i = member i (the same fp64 operations as the loop below)
  const int p0 = rl((int)h0.z, 0);
  const uint32_t cnt0 = wd_cnt(dj, p0);
  if (DGP_RUN_PAR && !ballot(lane < k && (int)h0.z != p0) && cnt0 > (uint32_t)k) {
    WDict di = dj;
    wd_set(di, p0, cnt0 - (uint32_t)(lane + 1));
    const double occ_i = occ_dict_r(di, nbw, durv, D);
    int64_t dnb = 0;
    if (lane < k) {
      SRec rc;
      rc.w = w;
      rc.p = (int16_t)p0;
      rc.kind = (int8_t)K_COMPLETE;
      rc.pad = 0;
      rc.nproc = np - (lane + 1);
      rc.task = (int)h0.x;
      rc.dnet = 0;
      rc.occ = occ_i;
      rc.dur = mkd(h2.x, h2.y);
      D.srec[(size_t)((r + lane) & (RS - 1)) * PLC] = rc;
      // add_replica (:3148) and the release of a dependency held by w (:3309-3314): integers
      dnb = ((h0.w & F_SELFREL) ? 0 : mk64(h1.x, h1.y)) - (((h1.z >> 8) & 0xff) ? mk64(er.z, er.w) : 0);
    }
    nbj += wsum64(dnb);
    wd_set(dj, p0, cnt0 - (uint32_t)k);
    np -= k;
  } else
  for (int i = 0; i < k; i++) {
    const int t = rl((int)h0.x, i), p = rl((int)h0.z, i);
    const uint32_t fl = rlu(h0.w, i);
    const int64_t nbt = mk64(rlu(h1.x, i), rlu(h1.y, i));
    const int nrel = (rlu(h1.z, i) >> 8) & 0xff;
    const double dobs = mkd(rlu(h2.x, i), rlu(h2.y, i));
    // processing -> memory: remove_from_processing, then the completion record (:2366)
    dict_add(dj, p, -1);
    np -= 1;
    Out o;
    o.nrec = 0;
    o.npl = 0;
    o.st0 = (size_t)((r + i) & (RS - 1)) * PLC;
    o.rec(D, K_COMPLETE, w, p, 0, occ_dict_r(dj, nbw, durv, D), np, t, dobs);
    // add_replica (:3148) and the release of a dependency held by w (:3309-3314)
    nbj += (fl & F_SELFREL) ? 0 : nbt;
    if (nrel) nbj -= mk64(rlu(er.z, i), rlu(er.w, i));
  }
  if (lane == 0) {
    using U4 = typename WPtr<LW>::template P<Q4>;
    P.nproc[w] = np;
    st4(ascast<U4>(P.pcnt + (size_t)w * PD), dj.c);
    st4(ascast<U4>(P.pcnt + (size_t)w * PD + 4), dj.c1);
    P.plen[w] = dj.ord;
    P.nbytes[w] = nbj;
  }
  if (n_dec && lane == d_ml) P.needs[(size_t)w * NLW + d_ml] = nl - (uint32_t)n_dec;
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): w's state is in LDS
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  // one release of w for the run: the stimulus after it on w counted one of the run's bits
  SMask bits = 0;
  for (int i = 0; i < k; i++) bits |= 1ull << rl(my_slot, i);
  if (lane == 0)
    release_succ(L, __hip_atomic_fetch_and(&P.mask[w], ~bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & ~bits);
  // retire every member: counts, then done, then the slots are free
  const int q = (int)((r + lane) & (RS - 1));
  if (lane < k) {
    RMeta me;
    me.npl = 0;
    me.nrec = 1;
    me.npops = 0;
    me.direct = 0;
    me.pad = 0;
    L.rmeta[q] = me;
  }
  __threadfence_block();
  if (lane < k) vstore(&L.rdone[q], r + lane + 1);
  if (lane == 0) atomicOr(&S.freem, bits);
  PROF(if (lane == 0) { S.prof[11] += 1; S.prof[12] += k; });
  return true;
}

// out of line, one register allocation each (inlined into the claim loop together they
// spilled to scratch)
template <bool LW>
__device__ __attribute__((noinline)) bool exe_run_entry(int s, long long r, uint4 E) {
  return exe_run<LW>(c_dev, st_L(), wptr<LW>(c_dev), s, r, E);
}

// wave argmin over all workers of a key computed per worker (global stimuli)
template <class F>
__device__ __forceinline__ Key argmin_workers(const Dev& D, F&& key_of) {
  const int lane = lane_id();
  Key best{INFINITY, INT64_MAX, INT32_MAX, 0};
  for (int c0 = 0; c0 < D.W; c0 += 64) {
    const int c = min(c0 + lane, D.W - 1);
    Key k;
    const bool ok = key_of(c, k) && c0 + lane < D.W;
    if (ok && key_less(k, best)) best = k;
  }
  for (int o = 32; o > 0; o >>= 1) {
    Key q;
    q.start = __shfl_xor(best.start, o);
    q.nb = __shfl_xor(best.nb, o);
    q.w = __shfl_xor(best.w, o);
    q.comm = __shfl_xor(best.comm, o);
    if (key_less(q, best)) best = q;
  }
  return best;
}

// A chunk of up to 64 frontier tasks (lane j: dependent j, `fr` set when stimulus r
// releases it) that all have ONE dependency, held by the same worker c, are not root-ish
// and share a prefix px already counted on c and in SchedulerState's global prefix dict
// (the P2P-shuffle unpack tasks of a barrier, shuffle/_shuffle.py:276-306): decide_worker
// returns c for each (:8579), comm is 0 and c needs no replica, so placement k differs from
// placement 0 only by the k earlier ones in c's count of px. Lane k evaluates placement k
// (start time from count + k, record from count + k + 1) with the serial path's exact
// expressions; the records fold in one walker batch. Returns false (nothing done) when the
// chunk does not qualify.
template <bool LW>
__device__ __attribute__((always_inline)) bool bulk_single_holder(const Dev& D, SCtl& S, const WPtr<LW>& P, WState& g,
                                                                  DTab durv, long long r, bool fr, int xl, int tfl,
                                                                  int h1l, long long lpos, int& npl) {
  const int lane = lane_id();
  const unsigned long long fm = ballot(fr);
  if (__builtin_popcountll(fm) < 2) return false;
  const int first = __builtin_ctzll(fm);
  const int c = rl(h1l, first);
  const int pxl = fr ? D.prefix[xl] : -1;
  const int px = rl(pxl, first);
  if (c < 0 || c >= D.W) return false;
  if (ballot(fr && (h1l != c || pxl != px || (tfl & TF_ROOTISH) || xl == D.dbg_task))) return false;
  const WDict d0 = dict_load<LW>(P, c);
  const uint32_t cnt0 = wd_cnt(d0, px);
  const bool in_g = ballot(lane < g.n && g.pf == px) != 0;
  if (cnt0 == 0 || !in_g) return false;
  const int m = __builtin_popcountll(fm);
  const int rank = __builtin_popcountll(fm & ((1ull << lane) - 1));
  const int np0 = P.nproc[c];
  const int64_t no0 = P.netocc[c], nb0 = P.nbytes[c];
  const double nth = (double)P.nthreads[c];
  // lane L: c's occupancy with L (before) and L + 1 (after) of these placements made
  WDict db = d0, da = d0;
  wd_set(db, px, cnt0 + (uint32_t)lane);
  wd_set(da, px, cnt0 + (uint32_t)lane + 1u);
  const double occ_b = occ_dict(db, no0, durv, D);
  const double occ_a = occ_dict(da, no0, durv, D);
  const double start_l = occ_b / nth + (double)(int64_t)0 / (double)D.bandwidth;  // place_x, comm = 0
  const double start = __shfl(start_l, rank);  // frontier lane -> its placement's start time
  if (fr) {
    const long long pos = lpos + npl + rank;
    D.pl_task[pos] = xl;
    D.pl_worker[pos] = c;
    D.pl_comm[pos] = 0;
    D.pl_start[pos] = start;
    D.pl_wsnbytes[pos] = nb0;
    D.pl_route[pos] = (int8_t)ROUTE_NONROOTISH;
    D.run_id[xl] = (int32_t)pos;
    D.holder_of[xl] = c;
    D.proc_on[xl] = c;
    D.state[xl] = S_PROCESSING;
    atomicAdd((unsigned long long*)&D.g_relwait[D.group[xl]], (unsigned long long)-1ll);
  }
  if (lane == 0) {
    using U4 = typename WPtr<LW>::template P<Q4>;
    WDict dn = d0;
    wd_set(dn, px, cnt0 + (uint32_t)m);
    st4(ascast<U4>(P.pcnt + (size_t)c * PD), dn.c);
    st4(ascast<U4>(P.pcnt + (size_t)c * PD + 4), dn.c1);
    P.nproc[c] = np0 + m;
  }
  __threadfence_block();
  // the m K_PLACE records in placement order (lane i = record i)
  SRec rc{};
  rc.w = c;
  rc.p = (int16_t)px;
  rc.kind = (int8_t)K_PLACE;
  rc.nproc = np0 + lane + 1;
  rc.task = -1;
  rc.dnet = 0;
  rc.occ = occ_a;
  rc.dur = 0.0;
  ws_fold_batch<LW>(D, P, S, g, rc, m);
  npl += m;
  return true;
}

// A chunk of frontier tasks that each have the same one dependency, the same prefix and the
// same ONE valid worker c, running (the shuffle's restricted unpacks: restrict_task shards
// the output partitions over the workers in contiguous ranges, so consecutive unpacks share
// their worker): decide_worker returns c for each (:8575-8586), placement k sees c with k of
// them made: count cnt0 + k of the prefix (its dict entry appended by the first if absent),
// the dependency's needs_what entry made by the first (netocc grows once) or counted up.
// The same operations as place_x one task at a time, lane L computing placement L.
template <bool LW>
__device__ __attribute__((always_inline)) unsigned long long bulk_restricted_same(const Dev& D, SCtl& S,
                                                                                  const WPtr<LW>& P, WState& g,
                                                                                  DTab durv, bool fr0, int from, int xl,
                                                                                  int rcl, int rdl, bool rhl,
                                                                                  int64_t rcml, bool evp,
                                                                                  long long lpos, int& npl) {
  // the run: the frontier lanes from lane `from` on, up to the first one that differs
  // (another worker, dependency or prefix); returns the lanes placed (0: none)
  const int lane = lane_id();
  const int first = from;
  const int c = rl(rcl, first), d = rl(rdl, first);
  const int pxl = fr0 ? D.prefix[xl] : -1;
  const int px = rl(pxl, first);
  const bool held = rl(rhl ? 1 : 0, first) != 0;
  const int64_t comm = rl_i64(rcml, first);
  if (c < 0 || c >= D.W || (evp && (P.wflags[c] & WF_PAUSED))) return 0;
  const unsigned long long diff = ballot(fr0 && lane >= from && (rcl != c || rdl != d || pxl != px || xl == D.dbg_task));
  const int lim = diff ? __builtin_ctzll(diff) : 64;
  const bool fr = fr0 && lane >= from && lane < lim;
  const unsigned long long fm = ballot(fr);
  const int m = __builtin_popcountll(fm);
  if (m < 2) return 0;
  WDict d0 = dict_load<LW>(P, c);
  const uint32_t cnt0 = wd_cnt(d0, px);
  if (cnt0 == 0 && wd_n(d0.ord) >= (uint32_t)PD) return 0;
  // the dependency's needs_what entry on c (lane i holds line word i)
  uint32_t nl = line_load<LW>(P, c);
  int64_t dnI = 0;  // netocc added by the first placement
  int ent = -1;
  bool ins = false;
  if (!held) {
    const uint32_t ctl = rlu(nl, NLW - 1);
    if (ctl == NL_OVF || (int)(ctl >> 8) != line_used(nl)) return 0;
    const unsigned long long hm = ballot(lane < NLW - 1 && nl != 0 && (nl >> 8) == (uint32_t)d);
    if (hm) {
      ent = __builtin_ctzll(hm);
      if ((rlu(nl, ent) & 0xffu) + (uint32_t)m > 0xffu) return 0;
    } else {
      const unsigned long long em = ballot(lane < NLW - 1 && nl == 0);
      if (!em) return 0;
      ent = __builtin_ctzll(em);
      ins = true;
      dnI = comm;  // _inc_needs_replica: the bytes c newly needs (:800-813), nbytes of d
    }
  }
  const int np0 = P.nproc[c];
  const int64_t no0 = P.netocc[c], nb0 = P.nbytes[c];
  const double nth = (double)P.nthreads[c];
  // lane L: placement L's occupancy before (count cnt0 + L; netocc grown after the first) and after
  WDict db = d0, da = d0;
  if (cnt0 + (uint32_t)lane > 0) wd_set(db, px, cnt0 + (uint32_t)lane);
  wd_set(da, px, cnt0 + (uint32_t)lane + 1u);
  const double occ_b = occ_dict(db, lane == 0 ? no0 : no0 + dnI, durv, D);
  const double occ_a = occ_dict(da, no0 + dnI, durv, D);
  const double start_l = occ_b / nth + (double)comm / (double)D.bandwidth;
  const int rank = __builtin_popcountll(fm & ((1ull << lane) - 1));
  const double start = __shfl(start_l, rank);
  if (fr) {
    const long long pos = lpos + npl + rank;
    D.pl_task[pos] = xl;
    D.pl_worker[pos] = c;
    D.pl_comm[pos] = comm;
    D.pl_start[pos] = start;
    D.pl_wsnbytes[pos] = nb0;
    D.pl_route[pos] = (int8_t)ROUTE_NONROOTISH;
    D.run_id[xl] = (int32_t)pos;
    D.holder_of[xl] = c;
    D.proc_on[xl] = c;
    D.state[xl] = S_PROCESSING;
    atomicAdd((unsigned long long*)&D.g_relwait[D.group[xl]], (unsigned long long)-1ll);
  }
  if (ent >= 0) {
    if (lane == ent) nl = ins ? (((uint32_t)d << 8) | (uint32_t)m) : nl + (uint32_t)m;
    if (ins && lane == NLW - 1) nl += 0x100u;
    line_store<LW>(P, c, nl);
  }
  if (lane == 0) {
    using U4 = typename WPtr<LW>::template P<Q4>;
    WDict dn = d0;
    wd_set(dn, px, cnt0 + (uint32_t)m);
    st4(ascast<U4>(P.pcnt + (size_t)c * PD), dn.c);
    st4(ascast<U4>(P.pcnt + (size_t)c * PD + 4), dn.c1);
    P.plen[c] = dn.ord;
    P.nproc[c] = np0 + m;
    P.netocc[c] = no0 + dnI;
  }
  __threadfence_block();
  SRec rc{};  // the m K_PLACE records in placement order (lane L = record L)
  rc.w = c;
  rc.p = (int16_t)px;
  rc.kind = (int8_t)K_PLACE;
  rc.nproc = np0 + lane + 1;
  rc.task = -1;
  rc.dnet = lane == 0 ? dnI : 0;
  rc.occ = occ_a;
  rc.dur = 0.0;
  ws_fold_batch<LW>(D, P, S, g, rc, m);
  npl += m;
  return fm;
}

// A chunk of frontier tasks that each have one dependency and ONE valid worker, running and
// different for every task of the chunk (the shuffle's restricted unpacks, range-sharded
// over the workers): decide_worker returns that worker (holders & valid, else valid,
// :8575-8586), and the placements touch disjoint workers, so each lane makes its task's
// placement on its own worker (occupancy before / after, the dict, needs_what, netocc, the
// log row) and the K_PLACE records are folded in placement order at once: the same
// operations as place_x one task at a time. False (nothing done) unless every frontier
// lane qualifies and every worker's dict and needs line take the change in place.
template <bool LW>
__device__ __attribute__((always_inline)) bool bulk_restricted_distinct(const Dev& D, SCtl& S, const WPtr<LW>& P,
                                                                        WState& g, DTab durv, bool fr, int xl, int rcl,
                                                                        int rdl, bool rhl, int64_t rcml, bool evp,
                                                                        long long lpos, int& npl) {
  const int lane = lane_id();
  const unsigned long long fm = ballot(fr);
  const int m = __builtin_popcountll(fm);
  if (m < 2) return false;
  bool ok = !fr || (rcl >= 0 && rcl < D.W && !(evp && (P.wflags[rcl] & WF_PAUSED)) && xl != D.dbg_task);
  if (ballot(!ok)) return false;
  bool dup = false;
  for (unsigned long long q = fm; q; q &= q - 1) {
    const int j = __builtin_ctzll(q);
    dup = dup || (fr && lane != j && rcl == rl(rcl, j));
  }
  if (ballot(dup)) return false;
  const int c = fr ? rcl : 0;
  const int px = fr ? D.prefix[xl] : 0;
  WDict dc = dict_load<LW>(P, c);
  const int np0 = P.nproc[c];
  const int64_t no0 = P.netocc[c], nb0 = P.nbytes[c];
  const double nth = (double)P.nthreads[c];
  int ent = -1;  // the needs_what entry of the dependency on c (-1: c holds it)
  bool ins = false;
  uint32_t ctl = 0, ev = 0;
  if (fr) {
    if (wd_find(dc, px) < 0 && wd_n(dc.ord) >= (uint32_t)PD) ok = false;
    if (!rhl) {
      ctl = P.needs[(size_t)c * NLW + NLW - 1];
      int used = 0, hit = -1, fz = -1;
      for (int i = 0; i < NLW - 1; i++) {
        const uint32_t e = P.needs[(size_t)c * NLW + i];
        used += e != 0 ? 1 : 0;
        if (e != 0 && (e >> 8) == (uint32_t)rdl) hit = i;
        if (e == 0 && fz < 0) fz = i;
      }
      if (ctl == NL_OVF || (int)(ctl >> 8) != used) {
        ok = false;
      } else if (hit >= 0) {
        ev = P.needs[(size_t)c * NLW + hit];
        if ((ev & 0xffu) == 0xffu) ok = false;
        ent = hit;
      } else if (fz >= 0) {
        ent = fz;
        ins = true;
      } else {
        ok = false;
      }
    }
  }
  if (ballot(!ok)) return false;
  const int rank = __builtin_popcountll(fm & ((1ull << lane) - 1));
  const int64_t dn = ins ? rcml : 0;  // _inc_needs_replica: the bytes c newly needs (:800-813)
  const double occ_b = occ_dict(dc, no0, durv, D);
  const double start = occ_b / nth + (double)rcml / (double)D.bandwidth;
  dict_add(dc, px, +1);
  const double occ_a = occ_dict(dc, no0 + dn, durv, D);
  if (fr) {
    const long long pos = lpos + npl + rank;
    D.pl_task[pos] = xl;
    D.pl_worker[pos] = c;
    D.pl_comm[pos] = rcml;
    D.pl_start[pos] = start;
    D.pl_wsnbytes[pos] = nb0;
    D.pl_route[pos] = (int8_t)ROUTE_NONROOTISH;
    D.run_id[xl] = (int32_t)pos;
    D.holder_of[xl] = c;
    using U4 = typename WPtr<LW>::template P<Q4>;
    st4(ascast<U4>(P.pcnt + (size_t)c * PD), dc.c);
    st4(ascast<U4>(P.pcnt + (size_t)c * PD + 4), dc.c1);
    P.plen[c] = dc.ord;
    P.nproc[c] = np0 + 1;
    P.netocc[c] = no0 + dn;
    if (ent >= 0) P.needs[(size_t)c * NLW + ent] = ins ? (((uint32_t)rdl << 8) | 1u) : ev + 1u;
    if (ins) P.needs[(size_t)c * NLW + NLW - 1] = ctl + 0x100u;
    D.proc_on[xl] = c;
    D.state[xl] = S_PROCESSING;
    atomicAdd((unsigned long long*)&D.g_relwait[D.group[xl]], (unsigned long long)-1ll);
  }
  __threadfence_block();
  // the records in placement order: frontier lane -> lane rank (lanes >= m unused)
  const int dst = (fr ? rank : 63) * 4;
  auto push = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)v); };
  SRec rc{};
  rc.w = (int)push((uint32_t)c);
  rc.p = (int16_t)push((uint32_t)px);
  rc.kind = (int8_t)K_PLACE;
  rc.nproc = (int)push((uint32_t)(np0 + 1));
  rc.task = -1;
  rc.dnet = mk64(push(lo32(dn)), push(hi32(dn)));
  rc.occ = mkd(push(dlo(occ_a)), push(dhi(occ_a)));
  rc.dur = 0.0;
  ws_fold_batch<LW>(D, P, S, g, rc, m);
  npl += m;
  return true;
}

// remove_all_replicas of a released dependency d (:3161-3171): every holder's ws.nbytes,
// then who_has = None (one lane per dependency; holders may be shared: LDS / global atomics)
template <bool LW>
__device__ __forceinline__ void release_replicas(const Dev& D, const WPtr<LW>& P, int d) {
  const int64_t nb = nbv(D, D.res_nbytes[d]);
  if ((D.evf & EVF_MULTI) && (D.tdyn[d] & TD_MULTI)) {
    for (int b = 0; b < D.WB; b++) {
      unsigned long long m = D.holders[(size_t)d * D.WB + b];
      D.holders[(size_t)d * D.WB + b] = 0;
      for (; m; m &= m - 1)
        __hip_atomic_fetch_add(P.nbytes + (b * 64 + __builtin_ctzll(m)), -nb, __ATOMIC_RELAXED,
                               LW ? __HIP_MEMORY_SCOPE_WORKGROUP : __HIP_MEMORY_SCOPE_AGENT);
    }
    D.tdyn[d] &= (uint8_t)~TD_MULTI;
  } else {
    const int hd = D.holder_of[d];
    __hip_atomic_fetch_add(P.nbytes + hd, -nb, __ATOMIC_RELAXED, LW ? __HIP_MEMORY_SCOPE_WORKGROUP : __HIP_MEMORY_SCOPE_AGENT);
    D.holders[(size_t)d * D.WB + (hd >> 6)] = 0;
  }
}

// a stimulus that reads SchedulerState-global state: every earlier stimulus has retired,
// every later one waits, the walker is caught up. Exact restatement of the whole
// transition (:2366-2442, :2313-2336, :4983-5023) for any route; placements go straight
// into the placement log, records are folded as they happen.
template <bool LW>
__device__ __attribute__((always_inline)) void exe_global(const Dev& D, SLds& L, const WPtr<LW>& P, int s, long long r) {
  SCtl& S = L.c;
  const int lane = lane_id();
  const uint4 E = lane < NE ? D.desc[(size_t)(r & (DR - 1)) * NE + lane] : make_uint4(0, 0, 0, 0);
  const DTab durv = stim_durations(D, L, E, r);
  const int t = rl((int)E.x, 0), w = rl((int)E.y, 0), p = rl((int)E.z, 0);
  const int64_t nbt = mk64(rlu(E.x, 1), rlu(E.y, 1));
  const int grp_t = rl((int)E.w, 1);
  const double dobs = mkd(rlu(E.x, 2), rlu(E.y, 2));
  WState g;
  ws_load(S, g);
  const long long lpos = S.log_len;
  int npl = 0;
  auto put_log = [&](int task, int wk, int64_t comm, double start, int64_t wsnb, int route) {
    if (lane == 0) {
      const long long pos = lpos + npl;
      D.pl_task[pos] = task;
      D.pl_worker[pos] = wk;
      D.pl_comm[pos] = comm;
      D.pl_start[pos] = start;
      D.pl_wsnbytes[pos] = wsnb;
      D.pl_route[pos] = (int8_t)route;
      D.run_id[task] = (int32_t)pos;
      D.holder_of[task] = wk;
    }
    npl++;
  };
  auto comm_bytes = [&](int x, int c) -> int64_t {  // worker_objective's sum :3136-3138
    int64_t v = 0;
    for (int64_t k = D.dep_ptr[x] + lane; k < D.dep_ptr[x + 1]; k += 64) {
      const int d = D.dep_idx[k];
      if (!holds_any(D, d, c)) v += nbv(D, D.res_nbytes[d]);
    }
    return wsum64(v);
  };
  const bool evp = (D.evf & EVF_PAUSED) != 0;
  auto paused = [&](int c) { return evp && (P.wflags[c] & WF_PAUSED); };
  // x's candidates need decide_worker's general form: a dependency with several replicas
  // (who_has row) or a paused holder (uniform; all lanes)
  auto gen_x = [&](int x) -> bool {
    if (!(D.evf & (EVF_MULTI | EVF_PAUSED))) return false;
    bool gx = false;
    for (int64_t q = D.dep_ptr[x] + lane; q < D.dep_ptr[x + 1]; q += 64) {
      const int d = D.dep_idx[q];
      const int h = D.holder_of[d];
      gx = gx || ((D.evf & EVF_MULTI) && (D.tdyn[d] & TD_MULTI)) || (h >= 0 && h < D.W && paused(h));
    }
    return ballot(gx) != 0;
  };
  WDict wd;
  bool skip_deps = false;  // the caller knows c holds every dependency of x
  // _add_to_processing (:3199) of x on c; x WAITING (frontier) or QUEUED (refill)
  auto place_x = [&](int x, int c, int route, int64_t comm, bool was_waiting) {
    if (comm < 0) comm = comm_bytes(x, c);
    const double oc = occ_of<LW>(P, D, c, durv);
    put_log(x, c, comm, oc / (double)P.nthreads[c] + (double)comm / (double)D.bandwidth, P.nbytes[c], route);
    const int px = D.prefix[x];
    const int np0 = P.nproc[c];
    const int64_t no0 = P.netocc[c];
    if (!dict_update<LW>(P, c, px, +1, wd)) serr(S, SERR_PREFIX, x);
    uint32_t nl = line_load<LW>(P, c);
    int64_t dn = 0;
    for (int64_t k = skip_deps ? 0 : D.dep_ptr[x]; !skip_deps && k < D.dep_ptr[x + 1]; k++) {
      if (rlu(nl, NLW - 1) == NL_OVF) {  // scan mode reads only: the rest lane-parallel
        dn += scan_needs_sum(D, k, D.dep_ptr[x + 1], c, x);
        break;
      }
      const int d = D.dep_idx[k];
      if (holds_any(D, d, c)) continue;
      dn += needs_inc(D, S, c, nl, d, nbv(D, D.res_nbytes[d]), x);
    }
    line_store<LW>(P, c, nl);
    if (lane == 0) {
      P.nproc[c] = np0 + 1;
      P.netocc[c] = no0 + dn;
      D.proc_on[x] = c;
      D.state[x] = S_PROCESSING;
      if (was_waiting) atomicAdd((unsigned long long*)&D.g_relwait[D.group[x]], (unsigned long long)-1ll);
    }
    __threadfence_block();
    ws_fold<LW>(D, P, S, g, K_PLACE, c, px, dn, occ_dict(wd, no0 + dn, durv, D), np0 + 1, 0.0);
  };
  auto itc_argmin = [&]() -> int {  // decide_worker_rootish_queuing_enabled :2230-2233
    Key b = argmin_workers(D, [&](int c, Key& k) {
      if (!D.sat_inf && (int)P.cap[c] - P.nproc[c] <= 0) return false;
      if (paused(c)) return false;  // idle_task_count holds running workers only (:2992)
      k.start = (double)P.nproc[c] / (double)P.nthreads[c];
      k.nb = 0;
      k.w = c;
      k.comm = 0;
      return true;
    });
    return b.w == INT32_MAX ? -1 : b.w;
  };
  bool queue_changed = false;
  // ------------------------------------------------------------- completion (:2366)
  {
    const int np0 = P.nproc[w];
    const int64_t no0 = P.netocc[w];
    // a long-running task left the prefix counts at add_to_long_running (:764-766)
    const bool lr = (D.evf & EVF_LR) && (D.tdyn[t] & TD_LR);
    if (lr) wd = dict_load<LW>(P, w);
    else dict_update<LW>(P, w, p, -1, wd);
    uint32_t nl = line_load<LW>(P, w);
    int64_t dnet = 0;
    for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
      if (rlu(nl, NLW - 1) == NL_OVF) {  // scan mode reads only: the rest lane-parallel
        dnet -= scan_needs_sum(D, k, D.dep_ptr[t + 1], w, t);
        break;
      }
      const int d = D.dep_idx[k];
      if (holds_any(D, d, w)) continue;
      dnet -= needs_dec(D, S, w, nl, d, nbv(D, D.res_nbytes[d]), t);
    }
    if (np0 - 1 == 0) needs_reset(D, w, nl);
    line_store<LW>(P, w, nl);
    if (lane == 0) {
      P.nproc[w] = np0 - 1;
      P.netocc[w] = no0 + dnet;
      P.nbytes[w] += nbt;  // add_replica :3148
      D.cur_nbytes[t] = nbt;
      D.proc_on[t] = -1;
      D.state[t] = S_MEMORY;
      if (lr) {  // long_running.discard: the slot it held on top of the cap goes
        P.cap[w] = (uint16_t)(P.cap[w] - 1);
        D.w_cap[w] -= 1;
        D.tdyn[t] &= (uint8_t)~TD_LR;
      }
    }
    __threadfence_block();
    ws_fold<LW>(D, P, S, g, lr ? K_COMPLETE_LR : K_COMPLETE, w, p, dnet, occ_dict(wd, no0 + dnet, durv, D),
                np0 - 1, dobs);
  }
  // ------------------------------------------------------ releases (:3309-3314, :2444)
  const int64_t f0 = D.dpt_ptr[t], f1 = D.dpt_ptr[t + 1];
  if (lane == 0) {
    if (f1 == f0 && !(D.tflags[t] & TF_WANTED)) {
      P.nbytes[w] -= nbt;
      D.state[t] = S_RELEASED;
      D.holders[(size_t)t * D.WB + (w >> 6)] = 0;
      atomicAdd((unsigned long long*)&D.g_relwait[grp_t], 1ull);
    }
    if constexpr (!LW) {
      for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
        const int d = D.dep_idx[k];
        if (D.rel_mark[d] != (int)r) continue;
        release_replicas<LW>(D, P, d);
        D.state[d] = S_RELEASED;
        atomicAdd((unsigned long long*)&D.g_relwait[D.group[d]], 1ull);
      }
    }
  }
  if constexpr (LW) {  // 64 deps at a time; holders' ws.nbytes by LDS atomics (int64: exact)
    lds_fence();
    for (int64_t k = D.dep_ptr[t] + lane; k < D.dep_ptr[t + 1]; k += 64) {
      const int d = D.dep_idx[k];
      if (D.rel_mark[d] != (int)r) continue;
      release_replicas<LW>(D, P, d);
      D.state[d] = S_RELEASED;
      atomicAdd((unsigned long long*)&D.g_relwait[D.group[d]], 1ull);
    }
    lds_fence();
  }
  wbar();
  // -------------------------------------- frontier, ascending priority (:2313-2336)
  // 64 dependents at a time: lane j prefetches dependent j's id, frontier mark, flags and,
  // for a single-dependency task, that dependency's holder (none of these change while
  // the frontier is placed), so the serial walk below reads them with readlane.
  bool fr_stop = false;
  for (int64_t k0 = f0; k0 < f1 && !fr_stop; k0 += 64) {
   int xl = 0, fml = -1, tfl = 0, h1l = -1;
   int rcl = -1;        // a restricted task with one dependency and one valid worker: that worker,
   int64_t rcml = 0;    // its comm bytes (the shuffle's restricted unpacks), the dependency
   int rdl = -1;        // and whether the worker holds it
   bool rhl = false;
   if (k0 + lane < f1) {
     xl = D.dpt_idx[k0 + lane];
     fml = D.fr_mark[xl];
     tfl = D.tflags[xl];
     const int64_t a = D.dep_ptr[xl], e = D.dep_ptr[xl + 1];
     if (e - a == 1 && !restricted_nonrootish(D, xl)) {
       const int d1 = D.dep_idx[a];
       h1l = D.holder_of[d1];
       // a replica set or a paused holder: decide_worker's general form below
       if (((D.evf & EVF_MULTI) && (D.tdyn[d1] & TD_MULTI)) || (h1l >= 0 && h1l < D.W && paused(h1l))) h1l = -1;
     } else if (e - a == 1 && restricted_nonrootish(D, xl) && restr_row(D, xl).r1 - restr_row(D, xl).r0 == 1) {
       const int d1 = D.dep_idx[a];
       if (!((D.evf & EVF_MULTI) && (D.tdyn[d1] & TD_MULTI))) {
         const RRow rr = restr_row(D, xl);
         rcl = rr.idx[rr.r0];
         rdl = d1;
         rhl = D.holder_of[d1] == rcl;
         rcml = rhl ? 0 : nbv(D, D.res_nbytes[d1]);
       }
     }
   }
   const int nk = (int)min((int64_t)64, f1 - k0);
   if (bulk_single_holder<LW>(D, S, P, g, durv, r, k0 + lane < f1 && fml == (int)r, xl, tfl, h1l, lpos, npl))
     continue;  // the whole chunk went to one worker, placed lane-parallel
   if (DGP_BULK_RESTR && bulk_restricted_distinct<LW>(D, S, P, g, durv, k0 + lane < f1 && fml == (int)r, xl, rcl, rdl,
                                                      rhl, rcml, evp, lpos, npl))
     continue;  // one task per worker, each on its own worker, lane-parallel
   const bool frl = k0 + lane < f1 && fml == (int)r;
   for (int j = 0; j < nk; j++) {
    const int x = rl(xl, j);
    if (rl(fml, j) != (int)r) continue;
    const int rc1 = rl(rcl, j);
    if (DGP_BULK_RESTR && rc1 >= 0) {  // a run of restricted tasks on one worker from j on: lane-parallel
      const unsigned long long done = bulk_restricted_same<LW>(D, S, P, g, durv, frl, j, xl, rcl, rdl, rhl, rcml, evp,
                                                               lpos, npl);
      if (done) {
        j = 63 - __builtin_clzll(done);
        continue;
      }
    }
    if (rc1 >= 0 && rc1 < D.W && !paused(rc1) && x != D.dbg_task) {
      // decide_worker with one valid running worker (:8575-8586): the candidates are that
      // worker whether or not it holds the dependency (holders & valid, else valid)
      place_x(x, rc1, ROUTE_NONROOTISH, mk64(rlu(lo32(rcml), j), rlu(hi32(rcml), j)), true);
      continue;
    }
    if (restricted_nonrootish(D, x)) {
      // decide_worker (:8550-8593) with valid = valid_workers(ts) & running: candidates =
      // holders & valid; none: valid; valid empty: loose -> decide_worker without
      // restrictions (holders, else every running worker), else None -> no-worker
      const RRow rr = restr_row(D, x);
      const int64_t r0 = rr.r0, r1 = rr.r1;
      auto held = [&](int cw) {
        for (int64_t q = D.dep_ptr[x]; q < D.dep_ptr[x + 1]; q++)
          if (holds_any(D, D.dep_idx[q], cw)) return true;
        return false;
      };
      bool hv = false, av = false;
      for (int64_t i = r0 + lane; i < r1; i += 64) {
        const int cw = rr.idx[i];
        if (paused(cw)) continue;
        av = true;
        hv = hv || held(cw);
      }
      int mode = ballot(hv) ? 0 : ballot(av) ? 1 : (D.restr_flags[x] & RF_LOOSE) ? 2 : 4;
      Key b{INFINITY, INT64_MAX, INT32_MAX, 0};
      if (mode <= 1 && r1 - r0 <= 64) {  // the candidates are in the restriction row: one lane each
        const int cw = lane < r1 - r0 ? rr.idx[r0 + lane] : 0;
        const bool in = lane < r1 - r0 && !paused(cw) && (mode == 1 || held(cw));
        const double ocw = occ_of<LW>(P, D, cw, durv);
        if (in) {
          int64_t cm = 0;
          for (int64_t q = D.dep_ptr[x]; q < D.dep_ptr[x + 1]; q++)
            if (!holds_any(D, D.dep_idx[q], cw)) cm += nbv(D, D.res_nbytes[D.dep_idx[q]]);
          b.start = ocw / (double)P.nthreads[cw] + (double)cm / (double)D.bandwidth;
          b.nb = P.nbytes[cw];
          b.w = cw;
          b.comm = cm;
        }
        for (int o = 32; o > 0; o >>= 1) {
          Key q;
          q.start = __shfl_xor(b.start, o);
          q.nb = __shfl_xor(b.nb, o);
          q.w = __shfl_xor(b.w, o);
          q.comm = __shfl_xor(b.comm, o);
          if (key_less(q, b)) b = q;
        }
        mode = 5;  // decided
      }
      for (int tr = 0; tr < 2 && mode != 4 && mode != 5; tr++) {
        b = argmin_workers(D, [&](int cw, Key& kk) {
          const double ocw = occ_of<LW>(P, D, cw, durv);  // all lanes: it shuffles
          if (paused(cw)) return false;
          if (mode <= 1 && !restr_has(D, x, cw)) return false;
          if ((mode == 0 || mode == 2) && !held(cw)) return false;
          int64_t cm = 0;
          for (int64_t q = D.dep_ptr[x]; q < D.dep_ptr[x + 1]; q++)
            if (!holds_any(D, D.dep_idx[q], cw)) cm += nbv(D, D.res_nbytes[D.dep_idx[q]]);
          kk.start = ocw / (double)P.nthreads[cw] + (double)cm / (double)D.bandwidth;
          kk.nb = P.nbytes[cw];
          kk.w = cw;
          kk.comm = cm;
          return true;
        });
        if (b.w != INT32_MAX || mode != 2) break;
        mode = 3;  // every holder paused: every running worker
      }
      if (b.w == INT32_MAX) {  // -> no-worker (:2761-2782)
        if (lane == 0) {
          D.state[x] = S_NO_WORKER;
          atomicAdd((unsigned long long*)&D.g_relwait[D.group[x]], (unsigned long long)-1ll);
          D.ctl->n_unrunnable++;
        }
        __threadfence_block();
        continue;
      }
      place_x(x, b.w, ROUTE_NONROOTISH, b.comm, true);
      continue;
    }
    const int hx = rl(h1l, j);
    if (!(rl(tfl, j) & TF_ROOTISH) && hx >= 0 && hx < D.W && x != D.dbg_task) {
      // decide_worker (:8550-8593) with one dependency: its holder is the only candidate
      // and is returned directly (:8579); comm_bytes is 0 and c needs no new replica
      skip_deps = true;
      place_x(x, hx, ROUTE_NONROOTISH, 0, true);
      skip_deps = false;
      continue;
    }
    if (rl(tfl, j) & TF_ROOTISH) {
      const int gi = D.group[x];
      if (D.sat_inf) {  // decide_worker_rootish_queuing_disabled :2135-2193
        int c = D.g_lastw[gi];
        if (!(c >= 0 && D.g_left[gi] != 0 && !paused(c))) {  // lws.status == running (:2170)
          const bool use_idle = g.n_idle > 0;  // pool = idle or running (:2161)
          Key b = argmin_workers(D, [&](int cw, Key& kk) {
            const double ocw = occ_of<LW>(P, D, cw, durv);  // all lanes: it shuffles
            if (use_idle && !(P.wflags[cw] & WF_IDLE)) return false;
            if (!use_idle && paused(cw)) return false;
            int64_t cm = 0;
            for (int64_t q = D.dep_ptr[x]; q < D.dep_ptr[x + 1]; q++)
              if (!holds_any(D, D.dep_idx[q], cw)) cm += nbv(D, D.res_nbytes[D.dep_idx[q]]);
            kk.start = ocw / (double)P.nthreads[cw] + (double)cm / (double)D.bandwidth;
            kk.nb = P.nbytes[cw];
            kk.w = cw;
            kk.comm = cm;
            return true;
          });
          c = b.w;
          if (lane == 0)
            D.g_left[gi] = (int64_t)floor(((double)D.g_size[gi] / (double)D.total_nthreads) * (double)P.nthreads[c]);
        }
        if (lane == 0) {
          D.g_lastw[gi] = D.g_relwait[gi] > 1 ? c : -1;
          D.g_left[gi] -= 1;
        }
        wbar();
        place_x(x, c, ROUTE_ROOTISH_NOQ, -1, true);
      } else {  // decide_worker_rootish_queuing_enabled :2195-2245
        const int c = itc_argmin();
        if (c < 0) {  // -> queued (:2761): HeapSet.add, kept as a priority-sorted array
          if (lane == 0) {
            D.state[x] = S_QUEUED;
            atomicAdd((unsigned long long*)&D.g_relwait[gi], (unsigned long long)-1ll);
            long long lo = S.qhead, pos = S.qhead + S.qlen;
            const int64_t pr = D.prio[x];
            while (pos > lo && D.prio[D.qarr[pos - 1]] > pr) {
              D.qarr[pos] = D.qarr[pos - 1];
              pos--;
            }
            D.qarr[pos] = x;
            S.qlen++;
          }
          queue_changed = true;
          __threadfence_block();
        } else {
          place_x(x, c, ROUTE_ROOTISH_Q, -1, true);
        }
      }
    } else if (!gen_x(x) && D.dep_ptr[x + 1] > D.dep_ptr[x] && D.dep_ptr[x + 1] - D.dep_ptr[x] <= 64 &&
               x != D.dbg_task) {
      // decide_worker :8550-8593 with the candidates = the dependency holders held in
      // lanes (at most 64 deps): one objective per distinct holder instead of a sweep
      // over all W workers. Same keys and the same total order as the sweep below.
      const int64_t q0 = D.dep_ptr[x];
      const int kx = (int)(D.dep_ptr[x + 1] - q0);
      int hj = -1;
      int64_t nbj = 0;
      if (lane < kx) {
        const int d = D.dep_idx[q0 + lane];
        hj = D.holder_of[d];
        nbj = nbv(D, D.res_nbytes[d]);
      }
      bool first = lane < kx && hj >= 0 && hj < D.W;
      for (int j = 0; j < kx; j++) {
        const int hh = __shfl(hj, j);
        if (j < lane && hh == hj) first = false;
      }
      const unsigned long long fm = ballot(first);
      if (!fm) {
        serr(S, SERR_CAND, x);
        break;
      }
      const int cw = first ? hj : __shfl(hj, __builtin_ctzll(fm));
      const double ocw = occ_of<LW>(P, D, cw, durv);  // all lanes: it shuffles
      int64_t cm = 0;
      for (int j = 0; j < kx; j++) {
        const int hh = __shfl(hj, j);
        const int64_t nb = shfl64(nbj, j);
        if (hh != cw) cm += nb;
      }
      Key b{INFINITY, INT64_MAX, INT32_MAX, 0};
      if (first) {
        b.start = ocw / (double)P.nthreads[cw] + (double)cm / (double)D.bandwidth;
        b.nb = P.nbytes[cw];
        b.w = cw;
        b.comm = cm;
      }
      for (int o = 32; o > 0; o >>= 1) {
        Key q;
        q.start = __shfl_xor(b.start, o);
        q.nb = __shfl_xor(b.nb, o);
        q.w = __shfl_xor(b.w, o);
        q.comm = __shfl_xor(b.comm, o);
        if (key_less(q, b)) b = q;
      }
      place_x(x, b.w, ROUTE_NONROOTISH, b.comm, true);
    } else if (!gen_x(x) && D.dep_ptr[x + 1] - D.dep_ptr[x] > 64 && x != D.dbg_task) {
      // decide_worker :8550-8593 for a wide fan-in (the shuffle barrier: P deps): one
      // lane-parallel pass over the deps accumulates, per holder, the bytes it already
      // holds and how many deps it holds; then comm(c) = total - held(c) (exact int64)
      // and c is a candidate iff it holds one. Same keys as the sweep below.
      unsigned long long* HS = D.gw_held;
      unsigned long long* HC = D.gw_held + D.W;
      for (int c = lane; c < D.W; c += 64) {
        __hip_atomic_store(HS + c, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(HC + c, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __threadfence();
      int64_t tot = 0;
#if DGP_PROF_GLOBAL
      const unsigned long long tw0 = mclk();
#endif
      // 8 dependencies per lane per step: their loads are all in flight before the atomics
      // (one dependent chain dep_idx -> holder_of / res_nbytes per step, not per dependency)
      constexpr int UW = 8;
      const int64_t q1 = D.dep_ptr[x + 1];
      for (int64_t q0 = D.dep_ptr[x]; q0 < q1; q0 += 64 * UW) {
        int dq[UW], hq[UW];
        int64_t nq[UW];
#pragma unroll
        for (int u = 0; u < UW; u++) {
          const int64_t q = q0 + u * 64 + lane;
          dq[u] = q < q1 ? D.dep_idx[q] : -1;
        }
#pragma unroll
        for (int u = 0; u < UW; u++) {
          hq[u] = dq[u] >= 0 ? D.holder_of[dq[u]] : -1;
          nq[u] = dq[u] >= 0 ? nbv(D, D.res_nbytes[dq[u]]) : 0;
        }
#pragma unroll
        for (int u = 0; u < UW; u++) {
          tot += nq[u];
          if (hq[u] >= 0 && hq[u] < D.W) {
            __hip_atomic_fetch_add(HS + hq[u], (unsigned long long)nq[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(HC + hq[u], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      __threadfence();
#if DGP_PROF_GLOBAL
      PROF(if (lane == 0) S.prof[22] += mclk() - tw0);  // diagnostics: the wide fan-in's holder sums
#endif
      tot = wsum64(tot);
      Key b = argmin_workers(D, [&](int cw, Key& kk) {
        const double ocw = occ_of<LW>(P, D, cw, durv);  // all lanes: it shuffles
        const unsigned long long hc = __hip_atomic_load(HC + cw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int64_t hs = (int64_t)__hip_atomic_load(HS + cw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (hc == 0) return false;
        const int64_t cm = tot - hs;
        kk.start = ocw / (double)P.nthreads[cw] + (double)cm / (double)D.bandwidth;
        kk.nb = P.nbytes[cw];
        kk.w = cw;
        kk.comm = cm;
        return true;
      });
      if (b.w == INT32_MAX) {
        serr(S, SERR_CAND, x);
        break;
      }
      place_x(x, b.w, ROUTE_NONROOTISH, b.comm, true);
    } else if (D.dep_ptr[x + 1] > D.dep_ptr[x]) {  // decide_worker :8550-8593
      // candidates = who_has of the dependencies & running; none: every running worker
      // (valid_workers = running when a worker is paused, decide_worker_non_rootish :2262-2266)
      bool any_cand = true;
      auto key_x = [&](int cw, Key& kk) {
        const double ocw = occ_of<LW>(P, D, cw, durv);  // all lanes: it shuffles
        if (paused(cw)) return false;
        bool cand = !any_cand;
        for (int64_t q = D.dep_ptr[x]; q < D.dep_ptr[x + 1] && !cand; q++) cand = holds_any(D, D.dep_idx[q], cw);
        if (!cand) return false;
        int64_t cm = 0;
        for (int64_t q = D.dep_ptr[x]; q < D.dep_ptr[x + 1]; q++)
          if (!holds_any(D, D.dep_idx[q], cw)) cm += nbv(D, D.res_nbytes[D.dep_idx[q]]);
        kk.start = ocw / (double)P.nthreads[cw] + (double)cm / (double)D.bandwidth;
        kk.nb = P.nbytes[cw];
        kk.w = cw;
        kk.comm = cm;
        if (x == D.dbg_task) {
          double* B = D.dbgbuf + (size_t)lane * 8;
          B[0] = cw;
          B[1] = kk.start;
          B[2] = (double)kk.nb;
          B[3] = (double)cm;
          B[4] = ocw;
          B[5] = P.nproc[cw];
          B[6] = (double)P.netocc[cw];
          B[7] = (double)wd_n(P.plen[cw]) + 100.0 * r;
        }
        return true;
      };
      Key b = argmin_workers(D, key_x);
      if (b.w == INT32_MAX && evp) {  // every holder paused
        any_cand = false;
        b = argmin_workers(D, key_x);
      }
      if (b.w == INT32_MAX) {
        serr(S, SERR_CAND, x);
        break;
      }
      place_x(x, b.w, ROUTE_NONROOTISH, b.comm, true);
    } else {
      serr(S, SERR_CAND, x);
      break;
    }
   }
   if (vload(&S.error) != 0) fr_stop = true;
  }
  // ---------------------------- Scheduler.stimulus_queue_slots_maybe_opened :4983-5023
  if (S.qlen > 0 && !D.sat_inf) {
    long long slots = 0;
    for (int c = lane; c < D.W; c += 64) {
      const int a = (int)P.cap[c] - P.nproc[c];
      if (a > 0 && !paused(c)) slots += a;  // over idle_task_count (:5007-5010)
    }
    slots = wsum64(slots);
    for (long long k = 0; k < slots; k++) {
      if (S.qlen == 0) break;
      const int c = itc_argmin();
      if (c < 0) continue;
      const int q = D.qarr[S.qhead];
      wbar();
      if (lane == 0) {
        S.qhead++;
        S.qlen--;
      }
      wbar();
      place_x(q, c, ROUTE_ROOTISH_Q, 0, false);
    }
  }
  // the invariant local refills rely on, and whether queued tasks are interchangeable
  {
    bool open = false;
    for (int c = lane; c < D.W && !D.sat_inf; c += 64) open = open || ((int)P.cap[c] - P.nproc[c] > 0 && !paused(c));
    const bool any_open = ballot(open) != 0;
    if (lane == 0) S.inv_ok = (S.qlen == 0 || !any_open) ? 1 : 0;
    if (queue_changed) {
      const int p0 = S.qlen > 0 ? D.prefix[D.qarr[S.qhead]] : 0;
      bool bad = false;
      for (long long i = S.qhead + lane; i < S.qhead + S.qlen; i += 64) {
        const int q = D.qarr[i];
        bad = bad || D.prefix[q] != p0 || D.dep_ptr[q + 1] > D.dep_ptr[q];
      }
      const bool anyb = ballot(bad) != 0;
      if (lane == 0) {
        S.q_anon = anyb ? 0 : 1;
        S.q_prefix = p0;
      }
    }
  }
  ws_store(S, g);
  __threadfence_block();
  release_slot<LW>(D, L, P, s, true);
  Out o;
  o.nrec = 0;
  o.npl = npl;
  o.st0 = (size_t)(r & (RS - 1)) * PLC;
  finish_slot(D, L, s, r, o, 0, true);
  if (lane == 0) vstore(&S.global_pending, 0);
}

// the global path out of line: the local path keeps its own register budget
template <bool LW>
__device__ __attribute__((noinline)) void exe_global_entry(int s, long long r) {
  exe_global<LW>(c_dev, st_L(), wptr<LW>(c_dev), s, r);
}

// G: this executor also runs the global stimuli. Only one executor wave does: a call to the
// global path from the others' loop would make the compiler keep its clobbers out of their
// registers (measured: +18% on the C2 replay from spills in the claim loop). A global-only
// G wave (no second copy of exe_local) was measured slower: C2 1.18 -> 1.27 s.
template <bool LW, bool G>
__device__ __attribute__((always_inline)) void role_exe(const Dev& D, SLds& L, const WPtr<LW>& P) {
  SCtl& S = L.c;
  const int lane = lane_id();
  unsigned long long t_idle = mclk();
  // idle / gated ticks accumulate in registers (an LDS atomic per poll from every idle
  // executor contends with the working waves' LDS traffic); flushed once at exit
  unsigned long long idle28 = 0, idle29 = 0;
  // DGP_EXE_PF: the descriptor of the oldest registered stimulus still waiting for its
  // workers (slot pf_s), loaded while idle: the executor that claims it next has it in registers
  long long pf_r = -1;
  int pf_s = 0;
  uint4 pfE = make_uint4(0, 0, 0, 0);
  while (true) {
    if (vload(&S.stop)) break;
    const SMask m = vload(&S.ready);
    if (!m) {
      const unsigned long long n = mclk();  // 28: executor idle, nothing ready
      idle28 += n - t_idle;
      t_idle = n;
      if (DGP_EXE_PF && !(vload(&L.pred[pf_s]) > 0 && vload(&L.sid[pf_s]) == pf_r)) {
        const long long sp = vload(&S.seq_pos);
        const SMask fm = vload(&S.freem);
        const bool wl = lane < WIN && !((fm >> lane) & 1ull) && vload(&L.pred[lane]) > 0;
        const unsigned k = wl ? (unsigned)(((vload(&L.sid[lane]) - sp) << 6) | lane) : ~0u;
        const unsigned kmin = wmin_u32(k);
        if (kmin != ~0u) {
          pf_s = (int)(kmin & 63u);
          pf_r = sp + (long long)(kmin >> 6);
          pfE = lane < NE ? D.desc[(size_t)(pf_r & (DR - 1)) * NE + lane] : make_uint4(0, 0, 0, 0);
        }
      }
      __builtin_amdgcn_s_sleep(DGP_EXE_SLEEP);
      continue;
    }
    // the ready slots in stimulus order (oldest first): lane i holds slot i's key
    const long long sp = vload(&S.seq_pos);
    const bool rdl = lane < WIN && ((m >> lane) & 1ull);
    const long long rsl = rdl ? vload(&L.sid[lane]) : 0;
    const uint32_t fsl = rdl ? vload(&L.flags[lane]) : 0u;
    // WAITC: a stimulus whose candidates are final first (it never waits in place); the
    // global-capable executor takes no other
    const bool pcl = WAITC && rdl && vload(&L.predc[lane]) != 0;
    const bool pskip = pcl && (G || rsl - sp >= WAITC_AHEAD);
    unsigned key = rdl && !pskip ? (unsigned)((pcl ? 1u << 31 : 0u) | ((rsl - sp) << 6) | lane) : ~0u;  // r - sp < RS
    int cs = -1, cq = 0;
    long long cr = -1;
    uint32_t cf = 0;
    bool cex = false;
    uint4 E = make_uint4(0, 0, 0, 0);
    while (true) {
      const unsigned kmin = wmin_u32(key);
      if (kmin == ~0u) break;
      const int s = (int)(kmin & 63u);
      if (lane == s) key = ~0u;  // tried
      if (!G && (rlu(fsl, s) & (F_GLOBAL | F_RUNM))) continue;  // left to the global-capable executor
      // WAITC: the global-capable executor never waits in place (it takes only stimuli whose
      // candidates are final), so the oldest stimulus always finds an executor that runs it
      if (G && WAITC && vload(&L.predc[s]) != 0) continue;  // (went non-final since the scan: cannot; kept as a guard)
      // the descriptor of the slot's stimulus (global ring) is in flight while the claim completes
      const long long rs = (long long)rl64((uint64_t)rsl, s);
      if (DGP_EXE_PF && rs == pf_r) E = pfE;
      else E = lane < NE ? D.desc[(size_t)(rs & (DR - 1)) * NE + lane] : make_uint4(0, 0, 0, 0);
      // claim first, then read the slot: between the scan and the claim its stimulus may
      // have run and retired and the slot been registered again (another stimulus)
      SMask old = 0;
      if (lane == 0) old = atomicAnd(&S.ready, ~(1ull << s));
      old = rl64(old, 0);
      if (!((old >> s) & 1ull)) continue;
      lds_fence();
      const long long r = vload(&L.sid[s]);
      if (r != rs) E = lane < NE ? D.desc[(size_t)(r & (DR - 1)) * NE + lane] : make_uint4(0, 0, 0, 0);
      const uint32_t fl = vload(&L.flags[s]);
      bool exact = (fl & (F_GLOBAL | F_EXACT)) != 0;
      int qm = 0;  // 0 no refill, 1 every open slot is refilled, 2/3 the queue length decides
      const long long ql = vload(&S.qlen);
      const long long spn = vload(&S.seq_pos);
      if (!(fl & F_GLOBAL) && ql > 0) {
        qm = (ql - (r - spn) * (long long)S.capmax >= (long long)S.capmax) ? 1 : 2;
        if (qm == 2) exact = true;
      }
      bool ok = G || !(fl & F_GLOBAL);
      if (ok && exact) {
        if (spn != r) ok = false;
        else if ((fl & F_GLOBAL) && vload(&S.walk_pos) != vload(&S.rec_len)) ok = false;
        if (qm != 0) qm = 3;
      }
      if (!ok) {  // not runnable by this executor now: give the slot back
        if (lane == 0) atomicOr(&S.ready, 1ull << s);
        continue;
      }
      cs = s;
      cr = r;
      cf = fl;
      cq = qm;
      cex = exact;
      break;
    }
    if (cs < 0) {
      const unsigned long long n = mclk();  // 29: ready slots, none claimable (exact gating)
      idle29 += n - t_idle;
      t_idle = n;
      __builtin_amdgcn_s_sleep(DGP_EXE_SLEEP);
      continue;
    }
    lds_fence();
    if (DGP_EXE_PRIO) __builtin_amdgcn_s_setprio(3);  // busy: ahead of the polling waves
    if (lane == 0) atomicAdd(&S.busy_exe, 1);
    if (DGP_TRACE && lane == 0) {
      TR(cr, 2);
      trace_at(D, cr, 7, D.trace && cr >= D.trace_lo && cr < D.trace_lo + D.trace_n
                             ? (D.trace[(cr - D.trace_lo) * TSTR + 7] | ((unsigned long long)(threadIdx.x >> 6) << 24)) : 0);
    }
    const unsigned long long t0 = mclk();
    if (D.resident && lane == 0) S.t_role[3] = rclk();
    if (G && (cf & F_GLOBAL)) {
      exe_global_entry<LW>(cs, cr);
#if DGP_PROF_GLOBAL  // diagnostics: cycles in global stimuli instead of their count
      PROF(if (lane == 0) S.prof[9] += mclk() - t0);
#else
      PROF(if (lane == 0) S.prof[9]++);
#endif
    } else if (G && (cf & F_SIMPLE) && cq == 0 && !cex && exe_run_entry<LW>(cs, cr, E)) {
      // a run of single-worker completions, back to back (only this executor calls out of line)
    } else {
      int wk = -1;
      const int rc = exe_local<LW>(D, L, P, cs, cr, cq, cex, E, wk) ? wk : -2;  // inlined: the common case
      if (rc == -2 && lane == 0) {
        atomicOr(&L.flags[cs], F_EXACT);
        atomicOr(&S.ready, 1ull << cs);
        PROF(S.prof[10]++);
      }
    }
    if (lane == 0) {
      PROF(atomicAdd(&S.prof[5], mclk() - t0));
      if (D.resident) S.t_role[4] = rclk();
      atomicSub(&S.busy_exe, 1);
    }
    if (DGP_EXE_PRIO) __builtin_amdgcn_s_setprio(DGP_EXE_PRIO == 2 ? 0 : 1);  // polling again
    t_idle = mclk();
  }
  if (lane == 0) {
    PROF(atomicAdd(&S.prof[28], idle28));
    PROF(atomicAdd(&S.prof[29], idle29));
  }
}

// ======================================================================== kernel
// all threads: worker state between the engine's global arrays and the stream layout
template <bool LW>
__device__ __attribute__((always_inline)) void workers_io(const Dev& D, const WPtr<LW>& P, bool load) {
  for (int c = threadIdx.x; c < D.W; c += blockDim.x) {
    if (load) {
      P.nproc[c] = D.w_nproc[c];
      P.nthreads[c] = (uint16_t)D.w_nthreads[c];
      P.cap[c] = (uint16_t)D.w_cap[c];
      // engine layout (insertion-ordered pairs) -> WDict slots (prefix ids < PX on this path)
      const int n = D.w_plen[c];
      for (int q = 0; q < PD; q++)
        P.pcnt[(size_t)c * PD + q] = q < n ? ((uint32_t)D.w_pfx[(size_t)c * PMAX + q] << 24) |
                                                 ((uint32_t)D.w_pcnt[(size_t)c * PMAX + q] & 0xffffffu)
                                           : 0u;
      P.plen[c] = (uint32_t)n << 24;
      P.netocc[c] = D.w_netocc[c];
      P.nbytes[c] = D.w_nbytes[c];
      P.mask[c] = 0;
      P.wflags[c] = D.w_flags[c] & (WF_IDLE | WF_SAT | WF_PAUSED);
      // needs_what: the stream layout persists in gw_needs (the engine's lines stay unused)
      for (int i = 0; i < NLW; i++) P.needs[(size_t)c * NLW + i] = D.gw_needs_saved[(size_t)c * NLW + i];
    } else {
      D.w_nproc[c] = P.nproc[c];
      const uint32_t ord = P.plen[c];
      const int n = (int)wd_n(ord);
      D.w_plen[c] = n;
      for (int i = 0; i < PMAX; i++) {
        const uint32_t v = P.pcnt[(size_t)c * PD + i];
        D.w_pfx[(size_t)c * PMAX + i] = i < n ? (int)(v >> 24) : 0;
        D.w_pcnt[(size_t)c * PMAX + i] = i < n ? (int)(v & 0xffffffu) : 0;
      }
      D.w_netocc[c] = P.netocc[c];
      D.w_nbytes[c] = P.nbytes[c];
      const int slots = D.sat_inf ? 0 : (int)P.cap[c] - P.nproc[c];
      const bool itc = !(P.wflags[c] & WF_PAUSED) && (D.sat_inf || slots > 0);
      D.w_flags[c] = P.wflags[c] | (itc ? WF_ITC : 0);
      D.w_itcslots[c] = itc ? slots : 0;
      for (int i = 0; i < NLW; i++) D.gw_needs_saved[(size_t)c * NLW + i] = P.needs[(size_t)c * NLW + i];
    }
  }
}


// One call per role for the whole launch: each role is register-allocated on its own
// (inlined into one kernel body they shared one 128-VGPR budget and spilled to scratch
// on the executors' path).
template <bool LW>
__device__ __attribute__((noinline)) void entry_exe() { role_exe<LW, false>(c_dev, st_L(), wptr<LW>(c_dev)); }
template <bool LW>
__device__ __attribute__((noinline)) void entry_exe_g() { role_exe<LW, true>(c_dev, st_L(), wptr<LW>(c_dev)); }
template <bool LW>
__device__ __attribute__((noinline)) void entry_reg() { role_reg<LW>(c_dev, st_L(), wptr<LW>(c_dev)); }
template <bool LW>
__device__ __attribute__((noinline)) void entry_wlk() { role_wlk<LW>(c_dev, st_L(), wptr<LW>(c_dev)); }
template <int KIND>
__device__ __attribute__((noinline)) void entry_stage() { role_stage<KIND>(c_dev, st_L()); }

template <bool LW>
__global__ void __launch_bounds__(SCTA) k_stream(long long max_rounds, int snaps) {
  const Dev& D = c_dev;
  SLds& L = st_L();
  SCtl& S = L.c;
  const WPtr<LW> P = wptr<LW>(D);
  Ctl* c = D.ctl;
  Pos* pos = D.pos;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // ------------------------------------------------------------------ set-up
  workers_io<LW>(D, P, true);
  for (int i = tid; i < RS; i += blockDim.x) L.rdone[i] = -1;
  if (tid < WIN) {
    L.pred[tid] = BIG;
    L.flags[tid] = 0;
    L.ntouch[tid] = 0;
  }
  // run_id / holder of the placements this engine has not sequenced (update_graph's)
  for (long long i = pos->runid_upto + tid; i < (long long)c->n_placed; i += blockDim.x) {
    const int tk = D.pl_task[i];
    D.run_id[tk] = (int32_t)i;
    D.holder_of[tk] = D.pl_worker[i];
  }
  if (tid == 0) {
    L.bld_njobs = 0;
    S.stop = 0;
    S.error = 0;
    S.err_task = -1;
    S.global_pending = 0;
    S.busy_exe = 0;
    S.ready = 0;
    S.freem = ~0ull >> (64 - WIN);
    S.seq_pos = pos->seq;
    S.log_len = (long long)c->n_placed;
    S.rec_len = pos->rec_len;
    S.walk_pos = pos->walk;
    S.bld_pos = pos->bld;
    S.pre_pos = pos->pre;
    S.reg_pos = pos->reg;
    S.qhead = c->qhead;
    S.qlen = c->qlen;
    S.n_tasks = c->n_tasks;
    S.stim_end = D.svc ? *D.svc_len : -1;
    S.req_n = S.req_off = 0;
    S.req_pl0 = (long long)c->n_placed;
    S.req_seen = 0;
    S.round_end = D.svc ? S.stim_end : pos->round_end >= 0 ? pos->round_end : (long long)c->n_placed;
    S.rounds_left = max_rounds > 0 ? max_rounds : -1;
    S.prev_placed = pos->round_end >= 0 ? pos->prev_placed : (long long)c->n_placed;
    S.rounds_nonempty = c->rounds_nonempty;
    S.snaps = D.svc ? 0 : snaps;
    S.reg_limit = (!D.svc && (snaps || max_rounds > 0)) ? S.round_end : (1ll << 62);
    S.g_plen = min(c->g_plen, PG);
    for (int i = 0; i < PG; i++) {
      S.g_pfx[i] = i < c->g_plen ? c->g_pfx[i] : 0;
      S.g_pcnt[i] = i < c->g_plen ? c->g_pcnt[i] : 0;
    }
    S.g_netocc = c->g_netocc;
    for (int i = 0; i < PX; i++) S.wdur[i] = i < D.P ? D.pdur_walk[i] : -1.0;
    S.n_idle = c->n_idle;
    S.n_sat = c->n_sat;
    for (int i = 0; i < 32; i++) S.prof[i] = 0;
    S.capmax = 1;
    S.inv_ok = 1;
    S.q_anon = 1;
    S.q_prefix = 0;
  }
  __syncthreads();
  // queue metadata and the refill invariant (block reductions)
  {
    __shared__ int s_open, s_bad, s_cap;
    if (tid == 0) {
      s_open = 0;
      s_bad = 0;
      s_cap = 1;
    }
    __syncthreads();
    for (int w = tid; w < D.W; w += blockDim.x) {
      if (!D.sat_inf && (int)P.cap[w] - P.nproc[w] > 0 && !(P.wflags[w] & WF_PAUSED)) atomicOr(&s_open, 1);
      atomicMax(&s_cap, (int)P.cap[w]);
    }
    const int p0 = S.qlen > 0 ? D.prefix[D.qarr[S.qhead]] : 0;
    for (long long i = S.qhead + tid; i < S.qhead + S.qlen; i += blockDim.x) {
      const int q = D.qarr[i];
      if (D.prefix[q] != p0 || D.dep_ptr[q + 1] > D.dep_ptr[q]) atomicOr(&s_bad, 1);
    }
    __syncthreads();
    if (tid == 0) {
      S.capmax = s_cap;
      S.inv_ok = (S.qlen == 0 || !s_open) ? 1 : 0;
      S.q_anon = s_bad ? 0 : 1;
      S.q_prefix = p0;
    }
  }
  __threadfence_block();
  __syncthreads();
  // ------------------------------------------------------------------- roles
  long long round_start = pos->round_start_saved;
  // issue priority: the in-order registrar first, then the sequencer and executors; the
  // batch-tolerant builder / prefetcher / walker take the remaining issue slots
  if (wave == 3) __builtin_amdgcn_s_setprio(3);
  else if (wave == 0 || wave >= N_ROLE) __builtin_amdgcn_s_setprio(2);
  if (wave == 0) {
    if (pos->round_end < 0) round_start = 0;
    role_seq<LW>(D, L, P, round_start);
  } else if (wave == 1) {
    entry_stage<0>();
  } else if (wave == 2) {
    entry_stage<1>();
  } else if (wave == 3) {
    entry_reg<LW>();
  } else if (wave == 4) {
    entry_wlk<LW>();
  } else if (!((D.dbg >> 8) & 15) || wave - N_ROLE < ((D.dbg >> 8) & 15)) {  // dbg bits 8..11: executor count
    if (wave == N_ROLE) entry_exe_g<LW>();  // the executor that also runs global stimuli
    else entry_exe<LW>();
  }
  __threadfence_block();
  __syncthreads();
  // --------------------------------------------------------------- write-back
  workers_io<LW>(D, P, false);
  __shared__ long long s_itc, s_slots;
  if (tid == 0) {
    s_itc = 0;
    s_slots = 0;
  }
  __syncthreads();
  for (int w = tid; w < D.W; w += blockDim.x) {
    const int slots = D.sat_inf ? 0 : (int)P.cap[w] - P.nproc[w];
    if (!(P.wflags[w] & WF_PAUSED) && (D.sat_inf || slots > 0)) {
      atomicAdd((unsigned long long*)&s_itc, 1ull);
      atomicAdd((unsigned long long*)&s_slots, (unsigned long long)(long long)(D.sat_inf ? 0 : slots));
    }
  }
  __syncthreads();
  if (wave == 0 && lane == 0) {
    c->n_placed = (unsigned long long)S.log_len;
    c->qhead = S.qhead;
    c->qlen = S.qlen;
    c->n_tasks = S.n_tasks;
    c->n_itc = s_itc;
    c->itc_slots = s_slots;
    c->rounds_nonempty = S.rounds_nonempty;
    c->g_plen = S.g_plen;
    for (int i = 0; i < PG; i++) {
      c->g_pfx[i] = S.g_pfx[i];
      c->g_pcnt[i] = S.g_pcnt[i];
    }
    c->g_netocc = S.g_netocc;
    c->n_idle = S.n_idle;
    c->n_sat = S.n_sat;
    // the durations as of the last folded record (the walker drains the record log before
    // the launch ends): what the host-side snapshot and the next launch's globals read
    for (int i = 0; i < PX && i < D.P; i++) D.pdur_walk[i] = D.pdur_cur[i] = S.wdur[i];
    if (S.error && !c->error) {
      c->error = S.error;
      c->err_task = S.err_task;
    }
    for (int i = 0; i < 16; i++) c->prof2[i] = S.prof[i];
    if (S.error) {  // pipeline state for the post-mortem (dgp_stats wave_phase*)
      const int sl = 0;
      const long long dv[16] = {S.seq_pos, S.reg_pos, S.pre_pos, S.bld_pos, S.log_len,
                                (long long)S.ready, S.busy_exe, S.global_pending, (long long)L.flags[sl], L.pred[sl],
                                L.sid[sl], (long long)S.freem, S.walk_pos, S.rec_len, S.qlen, S.round_end};
      for (int i = 0; i < 16; i++) c->prof2[i] = (unsigned long long)dv[i];
    }
    for (int i = 0; i < 16; i++) c->prof[i < 8 ? i : 7] = i < 8 ? S.prof[16 + i] : c->prof[7];
    for (int i = 0; i < 8; i++) c->prof3[i] = S.prof[24 + i];
    pos->seq = S.seq_pos;

    pos->reg = S.reg_pos;
    pos->bld = S.bld_pos;
    pos->pre = S.pre_pos;
    pos->rec_len = S.rec_len;
    pos->walk = S.walk_pos;
    pos->runid_upto = S.log_len;
    pos->round_end = S.round_end;
    pos->round_start_saved = round_start;
    pos->prev_placed = S.prev_placed;
    c->rec_used = 0;
    c->walk_pos = 0;
  }
}

#if DGP_ST_PRIMARY  // the event kernels below do not depend on the window: defined once, in st
// ================================================================ steal confirmation
// WorkStealing.move_task_confirm, the "confirm" branch (stealing.py:376-384, the finally
// clause :396-399) on the engine state between launches (service mode): processing task t
// leaves its worker v (WorkerState.remove_from_processing :759-771: prefix counts, the
// needs_what of its dependencies -> network occupancy, _task_prefix_count_global) for the
// thief h (add_to_processing :733-745), then check_idle_saturated(h) and (v) (:2949-2995)
// with the current total occupancy. The task keeps its placement-log position as its run
// identity (the caller maps the new compute-task's run_id to it). One wave.
__global__ void __launch_bounds__(64) k_move_task(const Dev* __restrict__ Dp, int t, int h) {
  const Dev& D = *Dp;
  __shared__ SCtl S;  // needs_dec / needs_inc report inconsistencies through it
  const int lane = lane_id();
  if (lane == 0) {
    S.error = 0;
    S.err_task = -1;
    S.stop = 0;
  }
  __syncthreads();
  const int v = D.proc_on[t];
  if (D.state[t] != S_PROCESSING || v < 0 || v >= D.W || v == h) {
    if (lane == 0) set_error(D, ERR_BAD_STATE, t);
    return;
  }
  if (D.tdyn[t] & TD_LR) {  // long-running tasks leave the stealable bins (handle_long_running :5829-5831)
    if (lane == 0) set_error(D, ERR_UNSUPPORTED, t);
    return;
  }
  const int p = D.prefix[t];
  const int64_t k0 = D.dep_ptr[t], k1 = D.dep_ptr[t + 1];
  // victim: the dependencies it needed a replica of (not held there) are needed less
  uint32_t nl = lane < NLW ? D.gw_needs_saved[(size_t)v * NLW + lane] : 0u;
  int64_t freed = 0;
  for (int64_t k = k0; k < k1; k++) {
    const int d = D.dep_idx[k];
    if (holds_any(D, d, v)) continue;
    freed += needs_dec(D, S, v, nl, d, nbv(D, D.res_nbytes[d]), t);
  }
  const int npv = D.w_nproc[v] - 1;
  if (npv == 0) needs_reset(D, v, nl);
  if (lane < NLW) D.gw_needs_saved[(size_t)v * NLW + lane] = nl;
  // thief: a replica of each dependency it does not hold is needed
  uint32_t nh = lane < NLW ? D.gw_needs_saved[(size_t)h * NLW + lane] : 0u;
  int64_t added = 0;
  for (int64_t k = k0; k < k1; k++) {
    const int d = D.dep_idx[k];
    if (holds_any(D, d, h)) continue;
    added += needs_inc(D, S, h, nh, d, nbv(D, D.res_nbytes[d]), t);
  }
  if (lane < NLW) D.gw_needs_saved[(size_t)h * NLW + lane] = nh;
  __threadfence();
  if (lane == 0) {
    Ctl* c = D.ctl;
    wdict_dec(D, v, p);  // remove_from_processing: worker dict, then the global one
    D.w_nproc[v] = npv;
    D.w_netocc[v] -= freed;
    gdict_dec(D, p);
    if (!wdict_inc(D, h, p)) set_error(D, ERR_PREFIX_CAP, t);  // add_to_processing
    D.w_nproc[h] += 1;
    D.w_netocc[h] += added;
    if (!gdict_inc(D, p)) set_error(D, ERR_GPREFIX_CAP, t);
    c->g_netocc += (double)(added - freed);  // integers < 2^53: exact in any order
    D.proc_on[t] = h;
    D.holder_of[t] = h;
    for (int i = 0; i < 2; i++) {  // check_idle_saturated(thief), then (victim)
      const int w = i == 0 ? h : v;
      walk_flags(D, w, occupancy(D, w, D.pdur_walk), D.w_nproc[w]);
      itc_check(D, w, false);
    }
    if (S.error) set_error(D, S.error, S.err_task);
  }
}

// ============================================================= queue refill
// Scheduler.stimulus_queue_slots_maybe_opened (:4983-5023) on the engine state between
// launches (service mode), one wave: the open slots of idle_task_count summed before any
// transition (:5007-5012), then each takes the queue's head through
// _transition_queued_processing (:2797-2808) -> decide_worker_rootish_queuing_enabled
// (:2227-2236: argmin of len(processing) / nthreads over idle_task_count, lowest index on
// ties) -> _add_to_processing (:3199-3215: add_to_processing, check_idle_saturated,
// n_tasks). Returns the placements made (uniform).
__device__ long long refill_queue(const Dev& D, SCtl& S) {
  const int lane = lane_id();
  Ctl* c = D.ctl;
  // queue position and log length in registers (uniform); lane 0 writes them back at the end
  long long qhead = c->qhead, qlen = c->qlen, pos = (long long)c->n_placed;
  if (D.sat_inf || qlen <= 0) return 0;
  long long slots = 0;
  for (int i = lane; i < D.W; i += 64)
    if (D.w_flags[i] & WF_ITC) slots += (long long)D.w_cap[i] - D.w_nproc[i];
  slots = wsum64(slots);
  long long n = 0;
  for (long long k = 0; k < slots && qlen > 0; k++) {
    // decide_worker_rootish_queuing_enabled: argmin over idle_task_count
    double bk = INFINITY;
    int bi = INT32_MAX;
    for (int i = lane; i < D.W; i += 64) {
      if (!(D.w_flags[i] & WF_ITC)) continue;
      const double key = (double)D.w_nproc[i] / (double)D.w_nthreads[i];
      if (key < bk) {  // ascending index per lane: the first minimum stays
        bk = key;
        bi = i;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const double qk = __shfl_xor(bk, o);
      const int qi = __shfl_xor(bi, o);
      if (qk < bk || (qk == bk && qi < bi)) {
        bk = qk;
        bi = qi;
      }
    }
    if (bi == INT32_MAX) break;  // idle_task_count empty: the head stays queued
    const int ws = bi;
    const int t = D.qarr[qhead];
    // worker_objective's comm bytes (:3136-3138) and _inc_needs_replica (:800-813) of the
    // dependencies ws holds no replica of
    const int64_t k0 = D.dep_ptr[t], k1 = D.dep_ptr[t + 1];
    int64_t comm = 0, added = 0;
    uint32_t nl = lane < NLW ? D.gw_needs_saved[(size_t)ws * NLW + lane] : 0u;
    for (int64_t q = k0; q < k1; q++) {
      const int d = D.dep_idx[q];
      if (holds_any(D, d, ws)) continue;
      const int64_t nb = nbv(D, D.res_nbytes[d]);
      comm += nb;
      added += needs_inc(D, S, ws, nl, d, nb, t);
    }
    if (lane < NLW) D.gw_needs_saved[(size_t)ws * NLW + lane] = nl;
    __threadfence();
    __syncthreads();
    if (lane == 0) {
      const double stack = occupancy(D, ws, D.pdur_walk) / (double)D.w_nthreads[ws];
      D.pl_task[pos] = t;
      D.pl_worker[pos] = ws;
      D.pl_comm[pos] = comm;
      D.pl_start[pos] = stack + (double)comm / (double)D.bandwidth;
      D.pl_wsnbytes[pos] = D.w_nbytes[ws];
      D.pl_route[pos] = ROUTE_ROOTISH_Q;
      D.run_id[t] = (int32_t)pos;
      D.holder_of[t] = ws;
      D.state[t] = S_PROCESSING;
      D.proc_on[t] = ws;
      // WorkerState.add_to_processing (:733-745), the global prefix count, network occupancy
      const int p = D.prefix[t];
      if (!wdict_inc(D, ws, p)) set_error(D, ERR_PREFIX_CAP, t);
      D.w_nproc[ws] += 1;
      D.w_netocc[ws] += added;
      if (!gdict_inc(D, p)) set_error(D, ERR_GPREFIX_CAP, t);
      c->g_netocc += (double)added;
      walk_flags(D, ws, occupancy(D, ws, D.pdur_walk), D.w_nproc[ws]);
      itc_check(D, ws, false);
      c->n_tasks += 1;
      if (S.error) set_error(D, S.error, S.err_task);
    }
    __threadfence();  // the flags / counts above are read by every lane of the next scan
    __syncthreads();
    pos++;
    qhead++;
    qlen--;
    n++;
  }
  if (lane == 0) {
    c->n_placed = (unsigned long long)pos;
    c->qhead = qhead;
    c->qlen = qlen;
  }
  __threadfence();
  __syncthreads();
  return n;
}

// ===================================================================== worker joins
// Scheduler.add_worker (scheduler.py:4308-4441) on the engine state between launches
// (service mode). The host has grown every per-worker array to W and set the new worker
// w = W - 1's nthreads / cap; here: the empty WorkerState, check_idle_saturated(ws)
// (:4398), then stimulus_queue_slots_maybe_opened (:4416-4420, :4983-5023): the open slots
// of idle_task_count, each taking the queue's head through _transition_queued_processing
// (:2797-2808) -> decide_worker_rootish_queuing_enabled (:2227-2236: argmin of
// len(processing) / nthreads over idle_task_count, lowest index on ties) ->
// _add_to_processing (:3199-3215: add_to_processing, check_idle_saturated, n_tasks).
// bulk_schedule_unrunnable_after_adding_worker has nothing to schedule on this path (no
// restrictions: no task is no-worker). One wave; *placed = the placements made. The worker
// is w (its index in address order; the host opened its rows). A worker that joins paused
// (not in running, :4368-4369) is neither idle nor saturated nor in idle_task_count
// (check_idle_saturated :2980-2995) and takes no refill (:4416).
__global__ void __launch_bounds__(64) k_add_worker(const Dev* __restrict__ Dp, long long* placed, int w, int running) {
  const Dev& D = *Dp;
  __shared__ SCtl S;  // needs_inc reports inconsistencies through it
  const int lane = lane_id();
  if (lane == 0) {
    S.error = 0;
    S.err_task = -1;
    S.stop = 0;
    D.w_nproc[w] = 0;
    D.w_plen[w] = 0;
    D.w_netocc[w] = 0;
    D.w_nbytes[w] = 0;
    D.w_itcslots[w] = 0;
    D.w_lastcheck[w] = ~0ull;
    D.w_flags[w] = 0;
    *placed = 0;
  }
  for (int i = lane; i < PMAX; i += 64) {
    D.w_pfx[(size_t)w * PMAX + i] = 0;
    D.w_pcnt[(size_t)w * PMAX + i] = 0;
  }
  if (lane < NLW) D.gw_needs_saved[(size_t)w * NLW + lane] = 0;
  if (lane < NXW) D.gw_needs_ext[(size_t)w * NXW + lane] = 0;
  __threadfence();
  __syncthreads();
  if (!running) {
    if (lane == 0) D.w_flags[w] = WF_PAUSED;
    return;
  }
  if (lane == 0) {  // check_idle_saturated(ws): nothing processing -> idle; idle_task_count
    walk_flags(D, w, occupancy(D, w, D.pdur_walk), 0);
    itc_check(D, w, false);
  }
  __threadfence();
  __syncthreads();
  const long long n = refill_queue(D, S);
  if (lane == 0) *placed = n;
}

#endif  // DGP_ST_PRIMARY

}  // namespace DGP_ST_NS
}  // namespace dgp
