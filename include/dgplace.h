/* dgplace — MI355X-native placement engine for the dask.distributed scheduler hot path.
 *
 * C ABI of libdgplace.so (built from the HIP sources in distributed_amd/csrc for gfx950).
 * Plain pointers and sizes only; every call returns 0 on success or a negative
 * DGP_E* code, and dgp_last_error() describes the failure. Host buffers are
 * borrowed for the duration of the call. One engine = one device + one HIP
 * stream; calls must come from one host thread (the scheduler's event loop).
 *
 * Reference interfaces each entry point replaces (paths relative to
 * /root/reference/distributed/):
 *   dgp_set_workers       Scheduler.add_worker -> WorkerState(...) + check_idle_saturated
 *                         (scheduler.py:4308-4441, :4418)
 *   dgp_set_graph         Scheduler._create_taskstate_from_graph / _generate_taskstates
 *                         (scheduler.py:4512-4611, :4753): TaskState graph, priorities,
 *                         who_wants, TaskPrefix/TaskGroup membership, _rootish overrides
 *   dgp_update_graph      the update_graph stimulus: every runnable task recommended
 *                         "waiting" in priority order and transitioned (:4600-4651, :2045)
 *   dgp_tasks_finished    Scheduler.handle_task_finished (:5783-5797) for a batch of
 *                         task-finished messages, in arrival order: the checks of
 *                         stimulus_task_finished (:5025-5092), then for each accepted one
 *                         _transition(key, "memory") -> _transitions ->
 *                         stimulus_queue_slots_maybe_opened (:4983). Engine state stays
 *                         resident between calls (service mode)
 *   dgp_move_task         WorkStealing.move_task_confirm, "confirm" branch (stealing.py:333-399,
 *                         :376-384): a processing task moves from its worker to the thief
 *   dgp_add_worker        Scheduler.add_worker (scheduler.py:4308-4441): a worker joins a running
 *                         engine: total_nthreads (:4383), check_idle_saturated (:4398), the
 *                         queue refill stimulus_queue_slots_maybe_opened (:4416-4420)
 *   dgp_add_graph         a later Scheduler.update_graph on a running engine (scheduler.py:4662-4751,
 *                         _create_taskstate_from_graph :4512-4653): new tasks, then their
 *                         update_graph stimulus
 *   dgp_add_replicas      SchedulerState.add_replica (scheduler.py:3148-3153), e.g. from the
 *                         add-keys stream handler (Scheduler.add_keys :7359-7391)
 *   dgp_remove_replicas   SchedulerState.remove_replica (:3155-3159), e.g. from
 *                         release-worker-data (:5807-5815)
 *   dgp_set_worker_status Scheduler.handle_worker_status_change (:5850-5883)
 *   dgp_long_running      Scheduler.handle_long_running (:5817-5848)
 *   dgp_heartbeat         the placement inputs of Scheduler.heartbeat_worker: the bandwidth
 *                         EWMA (:4223-4226) and TaskPrefix.add_exec_time (:4247-4252, :972-975)
 *   dgp_set_worker_flags  idle / saturated membership set outside a placement (the stealing
 *                         extension's check_idle_saturated calls, stealing.py:396-399, :494-496)
 *   dgp_set_wanted        who_wants gaining / losing its last client (client_desires_keys
 *                         :5398-5415)
 *   dgp_task_erred        Scheduler.handle_task_erred (:5799-5805 -> stimulus_task_erred
 *                         :5094-5127)
 *   dgp_remove_worker     Scheduler.remove_worker's worker table (:5213-5231)
 *   dgp_lose_worker       the whole Scheduler.remove_worker stimulus (:5180-5303): processing
 *                         tasks released and re-placed, lost results recomputed (ABI 17),
 *                         with recompute chains in the scheduler's set orders
 *                         (dgp_lose_worker_ordered, ABI 21)
 *   dgp_sync_*            the scheduler's state after a stimulus it decided itself
 *   dgp_snapshot          one per-worker snapshot (occupancy, nbytes, processing, idle /
 *                         saturated / idle_task_count, queue length) at a caller-chosen point
 *   dgp_run_rounds        the synthetic executor of the replay protocol: round k completes
 *                         the tasks placed in round k-1 (tests/golden/gen_golden.py)
 *   dgp_get_placements    the compute-task decisions (_add_to_processing :3199 /
 *                         _task_to_msg :3421): task, worker, comm bytes, objective, route
 *   dgp_task_messages     the who_has / nbytes fields of their compute-task messages
 *                         (_task_to_msg :3421-3450)
 *   dgp_steal_balance     WorkStealing.steal_time_ratio (stealing.py:241-277) for every
 *                         processing task + one WorkStealing.balance() (:401-503, _get_thief
 *                         :532-542, move_task_request :279-331, check_idle_saturated)
 */
#ifndef DGPLACE_H
#define DGPLACE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DGP_ABI_VERSION 21

#define DGP_OK 0
#define DGP_E_ARG -1     /* invalid argument / shape */
#define DGP_E_HIP -2     /* HIP runtime error (no device, OOM, launch failure) */
#define DGP_E_STATE -3   /* call out of order (e.g. rounds before update_graph) */
#define DGP_E_DEVICE -4  /* the device engine detected an inconsistent state */
#define DGP_E_UNSUPPORTED -5  /* a case the engine leaves to the caller; nothing changed (ABI 16) */

/* placement routes (which reference decide_worker path produced it) */
#define DGP_ROUTE_NONROOTISH 0   /* decide_worker_non_rootish -> decide_worker (:2247, :8550) */
#define DGP_ROUTE_ROOTISH_Q 1    /* decide_worker_rootish_queuing_enabled (:2195) */
#define DGP_ROUTE_ROOTISH_NOQ 2  /* decide_worker_rootish_queuing_disabled (:2135) */
#define DGP_ROUTE_FASTPATH 3     /* no-dependency fast path of decide_worker_non_rootish (:2283-2305) */

/* task states (TaskState.state) */
#define DGP_RELEASED 0
#define DGP_WAITING 1
#define DGP_PROCESSING 2
#define DGP_QUEUED 3
#define DGP_NO_WORKER 4
#define DGP_MEMORY 5
#define DGP_ERRED 6

typedef struct dgp_engine dgp_engine;

int dgp_abi_version(void);

/* Create an engine on HIP device `device`. Returns NULL on failure (no device). */
dgp_engine* dgp_create(int device);
void dgp_destroy(dgp_engine* e);
const char* dgp_last_error(const dgp_engine* e);

/* distributed.scheduler.{bandwidth, default-data-size, unknown-task-duration,
 * worker-saturation} (distributed.yaml:13,16,28,24). saturation may be +inf. */
int dgp_set_config(dgp_engine* e, int64_t bandwidth, int64_t default_data_size, double unknown_duration,
                   double saturation);

/* Register n_workers running workers with the given thread counts (index = worker id). */
int dgp_set_workers(dgp_engine* e, int32_t n_workers, const int32_t* nthreads);

/* Upload the task graph (CSR dependencies, deduplicated). prio: unique sort keys of
 * TaskState.priority (smaller runs first). wanted: task has a client future.
 * rootish_override: -1 none, 0/1 = TaskState._rootish. Graph stays resident in HBM. */
int dgp_set_graph(dgp_engine* e, int64_t n_tasks, const int64_t* dep_ptr, const int32_t* dep_idx,
                  const int64_t* prio, const int32_t* prefix_id, int32_t n_prefixes,
                  const double* prefix_default_duration, const int32_t* group_id, int32_t n_groups,
                  const uint8_t* wanted, const int8_t* rootish_override);

/* Per-task completion reports used by dgp_run_rounds: output nbytes and the compute
 * startstops interval of the task-finished message. */
/* Worker restrictions of the graph's tasks (TaskState.worker_restrictions / host / resource
 * restrictions and loose_restrictions, scheduler.py:1338-1354, :4908-4922), each resolved
 * by the caller to its valid_workers set (:3043-3107) as ascending worker indices
 * (CSR restr_ptr[N+1] / restr_idx). flags[t] bit 0: restricted (a non-empty restriction
 * set; its valid set may be empty -> no-worker unless loose), bit 1: loose_restrictions.
 * Placement follows decide_worker_non_rootish / decide_worker (:2247-2311, :8550-8593):
 * restricted tasks are not root-ish (:2939) unless _rootish overrides. Null flags clear
 * them. After dgp_set_graph, before any stimulus; resets the engine. */
int dgp_set_restrictions(dgp_engine* e, const int64_t* restr_ptr, const int32_t* restr_idx, const uint8_t* flags);
/* Restrictions of n tasks changed while the graph runs: Scheduler.set_restrictions
 * (scheduler.py:7702-7707), which the P2P shuffle's restrict_task calls for each output
 * task (shuffle/_scheduler_plugin.py:101-115, :281-293). Task task[i] gets the valid workers
 * row_idx[row_ptr[i] .. row_ptr[i+1]) (ascending indices) and flags[i] (as above); its
 * root-ish flag follows (:2939). Between stimuli; keeps the engine's state. (ABI 12) */
int dgp_update_restrictions(dgp_engine* e, int64_t n, const int32_t* task, const int64_t* row_ptr,
                            const int32_t* row_idx, const uint8_t* flags);
/* TaskState._rootish of n tasks set while the graph runs (-1 None, 0 False, 1 True; is_rootish
 * :2929-2947): the shuffle plugin's _ensure_output_tasks_are_non_rootish sets False on the
 * barrier's dependents when the shuffle starts (shuffle/_scheduler_plugin.py:150-151,
 * :254-278). Between stimuli; keeps the engine's state. (ABI 12) */
int dgp_set_rootish(dgp_engine* e, int64_t n, const int32_t* task, const int8_t* value);
int dgp_set_task_results(dgp_engine* e, const int64_t* nbytes, const double* start, const double* stop);

/* Reset all dynamic state (tasks released, workers empty, placement log cleared). */
int dgp_reset(dgp_engine* e);

/* The update_graph stimulus. */
int dgp_update_graph(dgp_engine* e);

/* Run synthetic-executor rounds until no task is processing or max_rounds (<0: no
 * limit) rounds ran. *n_rounds_out receives the number of rounds executed. */
int dgp_run_rounds(dgp_engine* e, int64_t max_rounds, int64_t* n_rounds_out);

/* Answers to one task-finished message (status[i] of dgp_tasks_finished). */
#define DGP_TF_ACCEPTED 0        /* processing on that worker with that run_id: completed (:5090) */
#define DGP_TF_FREE_KEYS 1       /* forgotten / released / queued / no-worker, or a stale run from
                                    another worker: reply "free-keys" (:5036-5079) */
#define DGP_TF_ADD_KEYS 2        /* already in memory: Scheduler.add_keys (:5082-5083) */
#define DGP_TF_RELEASE 3         /* stale run_id from the worker it is processing on: the reference
                                    recommends "released" (:5080-5081); left to the caller */
#define DGP_TF_UNKNOWN_WORKER 4  /* worker index not registered (:5786-5787): ignored */
#define DGP_TF_IMPOSSIBLE 5      /* current run_id from another worker: the reference raises (:2398) */
#define DGP_TF_UNSUPPORTED 6     /* waiting -> memory (a result for a task that is waiting again) */

/* Service mode: a batch of task-finished messages (Scheduler.handle_task_finished), in
 * arrival order. Per message: task index, worker index, the run_id of the compute-task
 * message it answers (the placement-log position of that placement), nbytes (< 0: None)
 * and the "compute" startstop (start/stop NaN: no compute interval). status[i] receives
 * DGP_TF_*; the accepted ones run as stimuli in order. The batch crosses PCIe in one copy;
 * *n_new_placements receives how many placements the batch made (read them with
 * dgp_get_placements from the previous dgp_num_placements). */
int dgp_tasks_finished(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker, const int64_t* run_id,
                       const int64_t* nbytes, const double* start, const double* stop, int8_t* status,
                       int64_t* n_new_placements);

/* (ABI 19) The stream kernel's in-flight stimulus window for the launches from now on: 32
 * slots with wait-in-place claims (the default; the ordered C2 chain needs them) or 64 slots
 * without (graphs with worker restrictions or a wide frontier: their replay is window-bound,
 * DESIGN.md §9). Both builds live in this library and make identical placements; only speed
 * differs, so a caller may switch per graph (PlacementEngine does at load and at each later
 * graph). Ends a resident kernel (the next call relaunches it with the new window).
 * dgp_get_window returns the current one. */
int dgp_set_window(dgp_engine* e, int32_t window);
int dgp_get_window(dgp_engine* e);

/* Resident service mode (ABI 9): with `enabled`, dgp_tasks_finished keeps the stream kernel
 * launched between calls and hands it each batch through a mailbox in pinned host memory
 * (the kernel's sequencer answers the messages, runs their stimuli and copies the new
 * placements' task / worker back): no launch, no copy, no synchronisation per call. The
 * kernel ends by itself after 0.2 s without a request (the next call launches it again),
 * and every other entry point ends it first, so the calls keep their meaning; while it
 * runs, dgp_num_placements and dgp_get_placements of the last answer's placements (task /
 * worker columns only) read the mailbox. */
int dgp_set_resident(dgp_engine* e, int enabled);

/* (ABI 13) With `enabled`, every resident answer also carries the compute-task message
 * fields of its new placements (who_has / nbytes per dependency, as dgp_task_messages; the
 * kernel's sequencer writes them into the mailbox before it publishes the answer), and
 * dgp_task_messages of those placements reads the mailbox: no kernel stop, no launch, no
 * copy. Replaces the per-placement walk of SchedulerState._task_to_msg (scheduler.py
 * :3421-3450) over the dependencies' who_has sets for the extension's batches. */
int dgp_set_task_messages(dgp_engine* e, int enabled);

/* (ABI 15) dgp_tasks_finished in two halves, so that the caller's own work overlaps the
 * device's: _post takes the batch (arguments and checks as dgp_tasks_finished) and returns
 * as soon as the resident kernel has the request (launch per call: the batch is answered
 * here and the answer kept); _wait spins on the answer and returns what dgp_tasks_finished
 * would (status[i] for the posted n messages, *n_new_placements). In between, every entry
 * point that touches the device or the mailbox fails with DGP_E_STATE (the kernel is inside
 * the request); dgp_destroy waits for the answer. The extension posts a task-finished batch before it runs
 * the reference's Scheduler.handle_task_finished (scheduler.py:5783-5797) and waits at the
 * first decision that batch's transitions ask for (_transition_waiting_processing :2313,
 * _transition_queued_processing :2797): _transition_processing_memory's Python (:2366-2420)
 * runs while the device decides. */
int dgp_tasks_finished_post(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker,
                            const int64_t* run_id, const int64_t* nbytes, const double* start, const double* stop);
int dgp_tasks_finished_wait(dgp_engine* e, int8_t* status, int64_t* n_new_placements);

/* Steal confirmation (WorkStealing.move_task_confirm, stealing.py:333-399, its "confirm"
 * branch :376-384 and finally clause :396-399): processing task `task` leaves its worker
 * (the victim: WorkerState.remove_from_processing, scheduler.py:759-771) for `thief`
 * (add_to_processing :733-745): prefix counts, needs_what / network occupancy and the
 * scheduler-global prefix counts, then check_idle_saturated(thief) and (victim). The task
 * keeps its placement-log position as its run identity: its later task-finished message
 * comes from the thief with that run_id (dgp_tasks_finished). Service mode, graphs on the
 * stream engine (<= 32 prefixes); DGP_E_DEVICE if the task is not processing. */
int dgp_move_task(dgp_engine* e, int32_t task, int32_t thief);

/* A worker joins (Scheduler.add_worker, scheduler.py:4308-4441) with `nthreads` threads; its
 * index is the next one (W): the caller keeps the reference's worker order (addresses sorted,
 * SortedDict) equal to index order, so a joining worker's address sorts after the others.
 * On the device: the empty WorkerState, total_nthreads += nthreads (:4383; root-ish groups
 * re-evaluated, is_rootish :2929-2947), check_idle_saturated(ws) (:4398), then
 * stimulus_queue_slots_maybe_opened (:4416-4420, :4983-5023): queued tasks taken in queue
 * order by decide_worker_rootish_queuing_enabled (:2227-2236) onto idle_task_count.
 * *n_new_placements receives the placements made (read them with dgp_get_placements).
 * Service mode, graphs on the stream engine (<= 32 prefixes); refused (DGP_E_STATE) while a
 * task is no-worker (bulk_schedule_unrunnable_after_adding_worker :3173-3186 is not modelled).
 * Snapshots taken earlier read 0 for the new worker. */
int dgp_add_worker(dgp_engine* e, int32_t nthreads, int64_t* n_new_placements);
/* dgp_add_worker_at: Scheduler.add_worker (scheduler.py:4308-4441) for a worker whose address
 * sorts anywhere among the known ones: SchedulerState.workers is a SortedDict keyed by address
 * (:3746, the insertion :4353) and the engine's worker index is that order (the canonical
 * tie-break and the no-dependency round robin over workers.values(), :2286-2305). The new
 * worker takes index `position` (the number of engine workers, removed ones included, whose
 * address sorts before it); every worker index >= position held by the engine -- per-worker
 * state, holder_of / processing_on, who_has bitset columns, restriction rows, the groups'
 * last_worker -- moves up by one on the device. `running` 0: the worker joins paused (status
 * paused, :4368-4369): total_nthreads grows, it is neither running, idle, saturated nor in
 * idle_task_count, and no queue refill follows (:4416). dgp_add_worker(e, n, p) ==
 * dgp_add_worker_at(e, n, 1, W, p). Needs the stream engine settled (no stimulus prefetched
 * beyond the sequenced ones): true between service calls. */
int dgp_add_worker_at(dgp_engine* e, int32_t nthreads, int32_t running, int32_t position, int64_t* n_new_placements);

/* A later graph submission (Scheduler.update_graph, scheduler.py:4662-4751 ->
 * _create_taskstate_from_graph :4512-4653) on a running engine, service mode: n_new tasks
 * appended with indices N.. (dep_ptr / dep_idx relative to the new graph; dep_idx = -1 - t
 * names the earlier task t), priorities after every earlier task's (a new generation,
 * :4713), prefix / group ids in the engine-wide tables (n_prefixes / n_groups >= the
 * current counts; prefix_default_duration is read for the new prefixes only: a known
 * TaskPrefix keeps its duration average). Group sizes and root-ish groups follow the grown
 * graph (is_rootish :2929-2947). Then the update_graph stimulus of the new tasks (:4600-4651):
 * released -> waiting, the runnable ones to processing (or queued) in priority order.
 * *n_new_placements receives the placements made. Stream-engine graphs (<= 32 prefixes in
 * total); the earlier tasks keep their restrictions, the new ones have none.
 * A graph with dependencies on earlier tasks is appended (the dependents rows of those tasks
 * grow) but its update_graph stimulus is the scheduler's own (the earlier tasks' states
 * decide the new tasks' waiting_on, :4600-4651): the new tasks stay released, no placement is
 * made, and every stimulus call answers DGP_E_STATE until the caller hands over the
 * scheduler's state after that stimulus (dgp_sync_placements / _tasks / _workers / _globals,
 * below; the new tasks and the earlier tasks they depend on among the synced rows). */
int dgp_add_graph(dgp_engine* e, int64_t n_new, const int64_t* dep_ptr, const int32_t* dep_idx, const int64_t* prio,
                  const int32_t* prefix_id, int32_t n_prefixes, const double* prefix_default_duration,
                  const int32_t* group_id, int32_t n_groups, const uint8_t* wanted, const int8_t* rootish_override,
                  int64_t* n_new_placements);
/* dgp_add_graph whose update_graph stimulus is the scheduler's own whatever its dependencies
 * (the appended tasks stay released, dgp_sync_* must follow): a later graph whose tasks carry
 * restrictions (scheduler.py:4908-4922), which the caller hands over with
 * dgp_update_restrictions after the resync. (ABI 12) */
int dgp_add_graph_deferred(dgp_engine* e, int64_t n_new, const int64_t* dep_ptr, const int32_t* dep_idx,
                           const int64_t* prio, const int32_t* prefix_id, int32_t n_prefixes,
                           const double* prefix_default_duration, const int32_t* group_id, int32_t n_groups,
                           const uint8_t* wanted, const int8_t* rootish_override);
/* (ABI 16) The update_graph stimulus (Scheduler.update_graph :4662-4751 ->
 * _transition_released_waiting :2078-2119 -> decide_worker / queued) of the graph the last
 * dgp_add_graph_deferred appended, on the device: for a later graph whose tasks depend on
 * earlier ones (each earlier dependency in memory, or waiting / queued / processing: the new
 * task waits on it and it gains the new task as a waiter), carries worker restrictions (its
 * rows given first with dgp_update_restrictions) or outranks earlier tasks by user priority
 * (every task's rank given first with dgp_set_priorities; new root-ish tasks queue in their
 * priority place). Ends the pending state of the append (no dgp_sync_* needed). An earlier
 * dependency that is released, erred or forgotten (recomputed or failed by the scheduler,
 * :2082-2097) returns DGP_E_UNSUPPORTED with nothing changed: the scheduler decides that
 * stimulus and the caller resynchronises as before. Replaces the scheduler's Python for that
 * stimulus (scheduler.py:4600-4653). */
int dgp_graph_stimulus(dgp_engine* e, int64_t* n_new_placements);
/* dgp_release_tasks (ABI 21): client-releases-keys (scheduler.py:5417-5430). task[i]: every
 * task its transitions reach -- the released / forgotten keys (_client_releases_keys
 * :3400-3419), the dependencies they release or forget in turn (_propagate_released
 * :3337-3357, _transition_waiting_released :2579-2604, _propagate_forgotten :3359-3398) -- in
 * the order the scheduler's recommendation dict runs them (distributed_amd/loss.py
 * release_plan). Each is applied by its state: memory -> released with its replicas;
 * processing -> released (it leaves its worker); waiting / queued / no-worker -> released
 * (waiting_on, queued, unrunnable); a cancelled task leaves its dependencies' waiters.
 * who_wants emptied; forget[i] != 0: forgotten (the row stays, released, out of every
 * dependents walk). Then the queue refill (:5430). *n_new_placements: its placements.
 * DGP_E_UNSUPPORTED with nothing changed for an erred or forgotten task (the scheduler
 * decides, then dgp_sync_*). */
int dgp_release_tasks(dgp_engine* e, int64_t n, const int32_t* task, const uint8_t* forget, int64_t* n_new_placements);
/* dgp_reschedule (ABI 21): Scheduler._reschedule (scheduler.py:7900-7924) of a processing task
 * -- transitions({key: "released"}): it leaves its worker (check_idle_saturated), is
 * recommended waiting when something needs it and placed again by decide_worker, through the
 * worker-loss recommendation machine. *n_new_placements: 0 or 1. DGP_E_UNSUPPORTED (a task
 * nobody needs: its release would release its dependencies) leaves the engine to be
 * resynchronised as after dgp_lose_worker; DGP_E_STATE (ERR_BAD_STATE) for a task that is not
 * processing. */
int dgp_reschedule(dgp_engine* e, int32_t task, int64_t* n_new_placements);
/* dgp_graph_stimulus_ordered (ABI 21): dgp_graph_stimulus, and an earlier dependency that is
 * released is recomputed (_transition_released_waiting :2101-2106, back to results in
 * memory): the runnable new tasks are recommended waiting in the dict's order (priority
 * descending, popped LIFO) and run through the worker-loss recommendation machine; the
 * scheduler's set orders the cascade follows come as order rows, as for
 * dgp_lose_worker_ordered (distributed_amd/loss.py graph_orders). An erred or forgotten
 * earlier dependency still returns DGP_E_UNSUPPORTED with nothing changed. */
int dgp_graph_stimulus_ordered(dgp_engine* e, int64_t n_order, const int32_t* order_task, const int8_t* order_kind,
                               const int64_t* order_ptr, const int32_t* order_idx, int64_t* n_new_placements);

/* (ABI 20) The task prefix table anew (the stream engine carries at most 32 prefixes; a
 * long-lived scheduler meets more: TaskPrefix objects per key_split name, scheduler.py:923-1031).
 * task_prefix: every task's slot in a table of n_prefixes (<= 32) live prefixes -- those of
 * the tasks released / waiting / queued / processing / no-worker and of the workers' and
 * the global task_prefix_count (:733-784, :1884-1903); a task of a prefix left out is in
 * memory / erred / forgotten and the engine never reads its slot. prefix_default_duration:
 * each slot's default-task-durations entry (-1: none). Replaces the PX-prefix ceiling of
 * dgp_add_graph for a session: the caller compacts the table when a later graph would pass
 * it. Pending until dgp_sync_workers + dgp_sync_globals bring the dicts, durations and
 * queue in the new numbering (as after dgp_add_graph_deferred). Between stimuli. */
int dgp_remap_prefixes(dgp_engine* e, int32_t n_prefixes, const int32_t* task_prefix,
                       const double* prefix_default_duration);

/* (ABI 14) Every task's priority anew (n_tasks entries, unique and topological): a later
 * graph submitted with a user priority that outranks earlier tasks (Scheduler.update_graph's
 * _set_priorities, scheduler.py:4934-4981: -user priority first in the tuple) — appended
 * with dgp_add_graph_deferred, then the merged ranks here, then dgp_sync_* as for any
 * deferred graph. The dependents rows (the frontier order of _add_to_memory) and the queue
 * are re-sorted in the new order. */
int dgp_set_priorities(dgp_engine* e, const int64_t* prio);

/* ---- Service events: the other placement-input stimuli of a live scheduler, in the order the
 * scheduler handles them, between dgp_tasks_finished calls. Stream-engine graphs (<= 32 prefixes);
 * DGP_E_STATE otherwise. A case the engine does not model returns
 * DGP_E_DEVICE ("a service event the engine does not model") and the caller hands placement
 * back to the scheduler. Those returning n_new_placements may refill the queue
 * (stimulus_queue_slots_maybe_opened :4983-5023): read the placements with dgp_get_placements. */

/* SchedulerState.add_replica(task, worker) for each pair, in order (WorkerState.add_replica
 * :825-838: the worker's needs_what entry goes, ws.nbytes grows, who_has gains the worker:
 * decide_worker's candidates and worker_objective's comm bytes / tie-break follow). The task
 * must be in memory; a worker already holding it is a no-op. A worker whose needs_what is in
 * scan mode (> 63 entries) is not modelled. */
int dgp_add_replicas(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker);

/* SchedulerState.remove_replica(task, worker) for each pair (WorkerState.remove_replica
 * :786-798). The last replica of a task (release-worker-data then releases it to recompute,
 * :5813-5815) is not modelled. */
int dgp_remove_replicas(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker);

/* Scheduler.handle_worker_status_change: running = 0 pauses the worker (it leaves running,
 * idle, idle_task_count and saturated: never a decide_worker candidate, its completions are
 * still accepted); running = 1 runs it again (check_idle_saturated, then the queue refill). */
int dgp_set_worker_status(dgp_engine* e, int32_t worker, int32_t running, int64_t* n_new_placements);

/* Scheduler.handle_long_running(task, compute_duration): the task's prefix duration average
 * takes compute_duration (NaN: None), WorkerState.add_to_long_running (:747-757: the prefix
 * counts, and _task_slots_available's slot :8765-8767), check_idle_saturated, the refill. */
int dgp_long_running(dgp_engine* e, int32_t task, double compute_duration, int64_t* n_new_placements);

/* Scheduler.heartbeat_worker's placement inputs: SchedulerState.bandwidth after the EWMA (a
 * float from now on: comm and network terms divide by it) and TaskPrefix.add_exec_time for
 * each executing task's prefix, in message order (max_exec_time; a duration above twice the
 * duration average resets it to -1, so _calc_occupancy uses 2 max_exec_time). */
int dgp_heartbeat(dgp_engine* e, double bandwidth, int64_t n, const int32_t* prefix, const double* duration);

/* idle / saturated membership of the given workers as the scheduler holds it (a paused worker
 * is neither). */
int dgp_set_worker_flags(dgp_engine* e, int64_t n, const int32_t* worker, const uint8_t* idle,
                         const uint8_t* saturated);

/* who_wants of each task non-empty (1) or empty (0): a wanted task is not released when its
 * last dependent completes (_add_to_memory :3309-3316). */
int dgp_set_wanted(dgp_engine* e, int64_t n, const int32_t* task, const uint8_t* wanted);

/* Scheduler.handle_task_erred for a current run with no retries left: the task errs, the tasks
 * waiting on it (and theirs, transitively) err, dependencies nobody waits for and no client
 * wants are released, the worker leaves processing (check_idle_saturated), the queue refill.
 * A cascade that would release a task not in memory (cancel processing or waiting work) is
 * not modelled (nothing changes). */
int dgp_task_erred(dgp_engine* e, int32_t task, int64_t* n_new_placements);

/* ---- Resynchronisation. A stimulus the engine does not model is decided by the scheduler's
 * own Python (the extension hands that one stimulus back); afterwards the host passes the
 * scheduler's state and the engine continues from it. In this order:
 *   dgp_sync_placements  the placements the scheduler made meanwhile, appended to the placement
 *                        log (_add_to_processing :3199: task, worker, worker_objective's comm
 *                        bytes and start time, ws.nbytes, route): their run identity for
 *                        dgp_tasks_finished is their log position
 *   dgp_sync_tasks       rows of tasks whose state changed: TaskState.state (0-6 as dgp_task_states,
 *                        7 = forgotten: left SchedulerState.tasks, :2853), len(waiting_on),
 *                        len(waiters), processing_on, nbytes (raw), long-running, who_wants
 *                        non-empty, who_has (CSR of worker indices)
 *   dgp_sync_workers     every worker: status (0 running, 1 paused, 2 removed: it keeps its
 *                        index and is never a candidate), len(processing), len(long_running),
 *                        task_prefix_count in insertion order (plen entries of prefix ids /
 *                        counts, <= 8, row stride 8), _network_occ, nbytes, idle / saturated
 *                        membership, needs_what (CSR of task indices and counts)
 *   dgp_sync_globals     SchedulerState.n_tasks, _network_occ_global,
 *                        _task_prefix_count_global (insertion order), queued (HeapSet order),
 *                        TaskPrefix.duration_average / max_exec_time per prefix, bandwidth, per
 *                        group states["released"] + states["waiting"],
 *                        last_worker_tasks_left and last_worker (-1: None)
 * dgp_remove_worker is the worker-table part of Scheduler.remove_worker (scheduler.py
 * :5213-5231: the worker leaves workers / running / idle / idle_task_count / saturated and
 * total_nthreads); the rest of that stimulus (its processing tasks released and re-placed,
 * lost results recomputed, :5233-5300) is the scheduler's, synchronised as above. */
int dgp_remove_worker(dgp_engine* e, int32_t worker);
/* dgp_lose_worker: Scheduler.remove_worker (scheduler.py:5180-5303) of a worker that still
 * has processing tasks or sole replicas, decided on the device: the worker leaves the tables,
 * every replica it holds is removed (held: ws.has_what in its order), and the recommendations
 * {processing[i]: released..., lost results: released...} run through the transitions
 * (processing -> released -> waiting, memory -> released -> waiting, waiting -> processing
 * with decide_worker), LIFO as SchedulerState._transitions pops them. processing: the
 * worker's tasks in the order the scheduler iterates ws.processing. The placements append to
 * the placement log (*n_new_placements); paused workers may be present (decide_worker's
 * candidates are then the running holders, or every running worker). DGP_E_UNSUPPORTED: the
 * cascade reaches a case the engine does not restate (a released dependency: see
 * dgp_lose_worker_ordered; a queued or no-worker dependent, a task nobody needs); after a refusal from the device the engine
 * takes the scheduler's state (dgp_sync_*) as after dgp_remove_worker. */
int dgp_lose_worker(dgp_engine* e, int32_t worker, int64_t n_processing, const int32_t* processing, int64_t n_held,
                    const int32_t* held, int64_t* n_new_placements);
/* dgp_lose_worker_ordered (ABI 21): dgp_lose_worker, and
 *  - a released dependency of a task the cascade re-waits is recomputed in turn
 *    (_transition_released_waiting :2101-2106: a chain of recomputes back to results still in
 *    memory); a no-worker waiter of a lost result is re-waited like a processing one;
 *  - killed[i] != 0 (NULL: none): processing[i] ran out of retries (KilledWorker, :5239-5265):
 *    processing -> erred at once in the processing loop (:2630-2720), its waiting dependents
 *    erred in turn (waiting -> released -> erred :2579-2605, :2507-2537) and a dependency in
 *    memory that nobody waits for any more released with its replicas (:2444-2505).
 * Where the recommendations' order follows a Python set, the caller passes the scheduler's
 * iteration order: rows i = 0..n_order-1, sorted by (order_task, order_kind), name
 * order_idx[order_ptr[i], order_ptr[i+1]) as order_task[i]'s dependencies (kind 0:
 * ts.dependencies, a permutation of its row), its waiters (kind 1: ts.waiters, dependents of
 * it) or its dependents (kind 2: ts.dependents); a task without a row iterates in index
 * order. dgp_lose_worker is this call with no rows and nothing killed. DGP_E_UNSUPPORTED as
 * there (a queued waiter of a lost result; an erred cascade that reaches a processing / queued
 * task or would release one that is not in memory; an erred or forgotten dependency). */
int dgp_lose_worker_ordered(dgp_engine* e, int32_t worker, int64_t n_processing, const int32_t* processing,
                            const int8_t* killed, int64_t n_held, const int32_t* held, int64_t n_order,
                            const int32_t* order_task, const int8_t* order_kind, const int64_t* order_ptr,
                            const int32_t* order_idx, int64_t* n_new_placements);
int dgp_sync_placements(dgp_engine* e, int64_t n, const int32_t* task, const int32_t* worker, const int64_t* comm_bytes,
                        const double* start_time, const int64_t* ws_nbytes, const int8_t* route);
int dgp_sync_tasks(dgp_engine* e, int64_t n, const int32_t* task, const uint8_t* state, const int32_t* remaining,
                   const int32_t* waiters, const int32_t* processing_on, const int64_t* nbytes,
                   const uint8_t* long_running, const uint8_t* wanted, const int64_t* holder_ptr,
                   const int32_t* holder_idx);
int dgp_sync_workers(dgp_engine* e, int32_t n_workers, const int8_t* status, const int32_t* nproc,
                     const int32_t* n_long_running, const int32_t* plen, const int32_t* prefix, const int32_t* count,
                     const int64_t* netocc, const int64_t* nbytes, const uint8_t* idle, const uint8_t* saturated,
                     const int64_t* needs_ptr, const int32_t* needs_task, const int32_t* needs_count);
int dgp_sync_globals(dgp_engine* e, int64_t n_tasks_counter, double network_occ_global, int32_t g_plen,
                     const int32_t* g_prefix, const int64_t* g_count, int64_t n_queued, const int32_t* queued,
                     const double* duration_average, const double* max_exec_time, double bandwidth,
                     const int64_t* group_released_waiting, const int64_t* group_left, const int32_t* group_last_worker);

/* Append one worker snapshot (needs dgp_enable_snapshots): round index = number of calls
 * (update_graph's snapshot is round 0). */
int dgp_snapshot(dgp_engine* e);

/* Placement log (run_id order). */
int64_t dgp_num_placements(dgp_engine* e);
int dgp_get_placements(dgp_engine* e, int64_t offset, int64_t count, int32_t* task, int32_t* worker,
                       int64_t* comm_bytes, double* start_time, int64_t* ws_nbytes, int8_t* route);

/* The compute-task message fields of placements [offset, offset + count)
 * (SchedulerState._task_to_msg, scheduler.py:3421-3450: who_has / nbytes of every
 * dependency), from the engine's state now: call it after the engine call that made the
 * placements and before the next stimulus, as _add_to_processing builds the message.
 * Per placement j its dependencies dep_ptr[j] .. dep_ptr[j+1]-1 (the graph's CSR order):
 * dep_task (task index), dep_nbytes (TaskState.nbytes as sent, -1: none reported), and their
 * who_has holder_ptr[k] .. holder_ptr[k+1]-1 in holder_idx (ascending worker index: every
 * replica once add-keys / dgp_add_replicas added some). *n_deps / *n_holders receive the row
 * counts; with dep_ptr NULL the call only sizes (then call again with dep_ptr[count + 1],
 * dep_task / dep_nbytes[n_deps], holder_ptr[n_deps + 1], holder_idx[n_holders]). Ends the
 * resident kernel (like every call but dgp_tasks_finished). */
int dgp_task_messages(dgp_engine* e, int64_t offset, int64_t count, int64_t* n_deps, int64_t* n_holders,
                      int64_t* dep_ptr, int32_t* dep_task, int64_t* dep_nbytes, int64_t* holder_ptr,
                      int32_t* holder_idx);

/* Per-round worker snapshots (state after update_graph and after each round). */
int dgp_enable_snapshots(dgp_engine* e, int64_t max_rounds);
int dgp_get_snapshots(dgp_engine* e, int64_t* n_rounds, int32_t* nplaced, double* occupancy, int64_t* ws_nbytes,
                      int32_t* nprocessing, uint8_t* idle, uint8_t* saturated, uint8_t* idle_task_count,
                      int32_t* nqueued);
int dgp_get_task_states(dgp_engine* e, uint8_t* state);

/* Device timing of the engine's kernels over the work since the last reset:
 * for kernel id k (0 frontier_release, 1 candidate_commbytes, 2 replay = the persistent
 * stream kernel, 3 update_graph)
 * total milliseconds (HIP events on the engine's stream) and launch count. */
int dgp_kernel_times(dgp_engine* e, double* ms, int64_t* launches, int32_t n);
int dgp_set_timing(dgp_engine* e, int enabled);

/* Engine counters: out[0] placements, [1] non-empty rounds, [2] deterministic-reservation
 * steps of the ordered commit, [3] stimuli that ran as global (in order, alone),
 * [4] record-log length, [5] record-log walker position, [6..13] commit-kernel phase
 * cycles (s_memtime): setup, local steps, global stimuli, finish, walker, longest step,
 * [14..37] stream-kernel probes, [38] resident requests answered, [39..41] their device
 * ticks (100 MHz) answering / running / publishing, [42..48] per request, when each role of
 * the stream kernel last finished a batch after the request was appended (builder,
 * prefetcher, registrar, executor claim, executor done, sequencer, walker), summed. */
int dgp_stats(dgp_engine* e, int64_t* out, int32_t n);
/* Measurement helper (host only, no engine): the longest chain of ordered stimuli of a
 * replay's placement log (stimulus r completes pl_task[r]; stimuli touching one worker are
 * ordered), from stimulus `first` on. bench.py's latency bound = depth x the measured
 * link latency. No reference counterpart (the reference runs one stimulus at a time). */
int dgp_conflict_depth(int64_t n_tasks, const int64_t* dep_ptr, const int32_t* dep_idx, const uint8_t* wanted,
                       int64_t n_pl, const int32_t* pl_task, const int32_t* pl_worker, int64_t first,
                       int64_t* depth, int64_t* n_touch);

/* WorkStealing: the cost level of every processing task (steal_time_ratio,
 * stealing.py:241-277; -1 = not stealable) and one balance() (:401-503) over a
 * scheduler state given as host arrays. Workers: nthreads, WorkerState.occupancy,
 * len(processing), ws.nbytes, membership of idle / saturated; the totals of
 * SchedulerState.total_occupancy / total_nthreads and the bandwidth. Processing tasks:
 * processing_on (victim), get_task_duration, prefix in fast_tasks, dependencies (CSR
 * into the data arrays). Data (dependencies): raw nbytes (get_comm_cost), get_nbytes()
 * (worker_objective, steal_time_ratio), who_has (CSR of worker ids). Tie-break: the
 * canonical one of the golden fixtures (worker index last; bins in ascending task id;
 * saturated in ascending worker id). Outputs: levels[T]; the ordered steal requests
 * (task, victim, thief, level, cost = compute + victim comm cost, victim / thief combined
 * occupancy as logged), capacity T; *n_steals; per-worker in-flight occupancy and task
 * deltas; idle / saturated membership after the call. Restrictions (nullable): each
 * task's valid_workers as worker indices (CSR restr_ptr[T+1] / restr_idx) and flags (bit 0
 * restricted, bit 1 loose): _get_thief (stealing.py:532-542) takes the valid thieves, the
 * loose retry over all thieves, or skips the task. The plugin's own state (nullable):
 * levels_in = the levels of its stealable bins (key_stealable; -1 = not in a bin; null:
 * computed by steal_time_ratio), inflight_*_in = in_flight_occupancy / in_flight_tasks
 * of unconfirmed steals (null: none); the in-flight outputs are then the new totals, and
 * checked_out[w] = 1 for each victim check_idle_saturated ran on (:498-500).
 * Kernel-time ids 4 (levels + bins),
 * 5 (thief argmin), 6 (balance walk). */
int dgp_steal_balance(dgp_engine* e, int32_t n_workers, const int32_t* nthreads, const double* occupancy,
                      const int32_t* nprocessing, const int64_t* ws_nbytes, const uint8_t* idle,
                      const uint8_t* saturated, double total_occupancy, int64_t total_nthreads, int64_t bandwidth,
                      int64_t n_tasks, const int32_t* victim, const double* duration, const uint8_t* fast,
                      const int64_t* dep_ptr, const int32_t* dep_idx, int64_t n_data, const int64_t* data_nbytes,
                      const int64_t* data_get_nbytes, const int64_t* holder_ptr, const int32_t* holder_idx,
                      const int64_t* restr_ptr, const int32_t* restr_idx, const uint8_t* restr_flags,
                      const int8_t* levels_in, const double* inflight_occupancy_in, const int32_t* inflight_tasks_in,
                      int8_t* levels, int32_t* st_task, int32_t* st_victim, int32_t* st_thief, int32_t* st_level,
                      double* st_cost, double* st_occ_victim, double* st_occ_thief, int64_t* n_steals,
                      double* inflight_occupancy, int32_t* inflight_tasks, uint8_t* idle_out, uint8_t* saturated_out,
                      uint8_t* checked_out);

/* dgp_steal_order: the next dgp_steal_load / dgp_steal_balance takes its tasks in ascending
 * (priority, arrival) instead of their input order (the order the bins are walked in,
 * stealing.py:441-461 with the canonical tie-break), sorted on the device; n_tasks must be
 * that call's n_tasks. The plugin keeps its task rows in arrival slots (no host sort per
 * balance() call). Outputs still index the tasks in input order. (ABI 18) */
int dgp_steal_order(dgp_engine* e, int64_t n_tasks, const int64_t* priority, const int64_t* arrival);
/* dgp_steal_balance in phases, for a balance() sharded over ranks (one engine per GPU):
 *   dgp_steal_load       the inputs of dgp_steal_balance; levels, bins and the initial
 *                        thief order; *n_stealable = tasks in a bin (stealing.py:220-239)
 *   dgp_steal_thief_rows the per-task precompute of _get_thief (stealing.py:532-542:
 *                        argmin of worker_objective over the initial thieves, comm costs,
 *                        dependency holders) for stealable positions [lo, hi)
 *   dgp_steal_pack_rows / dgp_steal_unpack_rows  positions [lo, hi) to / from a device
 *                        buffer of dgp_steal_row_bytes() each (the all-gathered record)
 *   dgp_steal_run        the ordered walk of balance() (:401-503) and the outputs of
 *                        dgp_steal_balance. Every position must hold its row first. */
int dgp_steal_load(dgp_engine* e, int32_t n_workers, const int32_t* nthreads, const double* occupancy,
                   const int32_t* nprocessing, const int64_t* ws_nbytes, const uint8_t* idle, const uint8_t* saturated,
                   double total_occupancy, int64_t total_nthreads, int64_t bandwidth, int64_t n_tasks,
                   const int32_t* victim, const double* duration, const uint8_t* fast, const int64_t* dep_ptr,
                   const int32_t* dep_idx, int64_t n_data, const int64_t* data_nbytes, const int64_t* data_get_nbytes,
                   const int64_t* holder_ptr, const int32_t* holder_idx, const int64_t* restr_ptr,
                   const int32_t* restr_idx, const uint8_t* restr_flags, const int8_t* levels_in,
                   const double* inflight_occupancy_in, const int32_t* inflight_tasks_in, int64_t* n_stealable);
int dgp_steal_thief_rows(dgp_engine* e, int64_t lo, int64_t hi);
int64_t dgp_steal_row_bytes(void);
int dgp_steal_pack_rows(dgp_engine* e, int64_t lo, int64_t hi, void* device_dst);
int dgp_steal_unpack_rows(dgp_engine* e, int64_t lo, int64_t hi, const void* device_src);
int dgp_steal_run(dgp_engine* e, int8_t* levels, int32_t* st_task, int32_t* st_victim, int32_t* st_thief,
                  int32_t* st_level, double* st_cost, double* st_occ_victim, double* st_occ_thief, int64_t* n_steals,
                  double* inflight_occupancy, int32_t* inflight_tasks, uint8_t* idle_out, uint8_t* saturated_out,
                  uint8_t* checked_out);

#ifdef __cplusplus
}
#endif
#endif /* DGPLACE_H */
