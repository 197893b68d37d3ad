// dgp_ingest.c — the extension's graph ingestion (f4): one C pass over the new TaskStates
// of an update_graph (scheduler.py:4753-4981 builds them; SchedulerPlugin.update_graph,
// diagnostics/plugin.py:74-109, hands them over) into the engine's per-task columns.
//
// graph_from_tasks (distributed_amd/ext.py) sorts the tasks by TaskState.priority and
// calls dgp_ingest_columns on that list. Per task it reads the attributes the engine's
// arrays need (dependencies, prefix, group, who_wants, _rootish and the three kinds of
// restrictions) with no Python frame and no allocation per task:
//   * dependency edges: each dependency's position in the list through a pointer hash map
//     (TaskState objects are identity-unique in SchedulerState.tasks); a dependency outside
//     the list (an earlier graph's task) is appended to ``misses`` and named -1 - its
//     position there, which graph_from_tasks resolves with the engine's key index;
//   * prefix / group ids in first-seen order (pointer maps), with the first task of each,
//     from which Python takes the objects (names, duration_average);
//   * wanted (truth of who_wants), _rootish (-1 None / 0 / 1), restriction flags (bit 0
//     worker, 1 host, 2 resource restrictions; valid_workers is resolved in Python for
//     those rows only).
// Built with gcc against the stable ABI (Py_LIMITED_API 3.9) and loaded with ctypes.PyDLL
// (the GIL stays held; a Python error raised here propagates), so one build serves the
// scheduler's interpreter whatever its minor version. Host bookkeeping only: placement
// decisions are the device engine's.
#define Py_LIMITED_API 0x03090000
#include <Python.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  uintptr_t* key;
  int32_t* val;
  size_t mask;
} PtrMap;

static int pm_init(PtrMap* m, size_t n) {
  size_t cap = 16;
  while (cap < 2 * n + 2) cap <<= 1;
  m->key = (uintptr_t*)calloc(cap, sizeof(uintptr_t));
  m->val = (int32_t*)malloc(cap * sizeof(int32_t));
  m->mask = cap - 1;
  return m->key && m->val ? 0 : -1;
}
static void pm_free(PtrMap* m) {
  free(m->key);
  free(m->val);
}
static inline size_t pm_slot(const PtrMap* m, uintptr_t k) {
  uint64_t h = (uint64_t)k * 0x9E3779B97F4A7C15ull;
  size_t i = (size_t)(h >> 17) & m->mask;
  while (m->key[i] && m->key[i] != k) i = (i + 1) & m->mask;
  return i;
}
// the id of k, inserting it as next (first seen) when absent; *is_new tells which
static inline int32_t pm_get_or_add(PtrMap* m, uintptr_t k, int32_t next, int* is_new) {
  size_t i = pm_slot(m, k);
  if (m->key[i]) {
    *is_new = 0;
    return m->val[i];
  }
  m->key[i] = k;
  m->val[i] = next;
  *is_new = 1;
  return next;
}
// keeps the load factor under 1/2 for n entries (rehash into a larger table)
static int pm_reserve(PtrMap* m, size_t n) {
  if (2 * n + 2 <= m->mask + 1) return 0;
  PtrMap m2;
  if (pm_init(&m2, n)) return -1;
  for (size_t s = 0; s <= m->mask; s++)
    if (m->key[s]) {
      const size_t k = pm_slot(&m2, m->key[s]);
      m2.key[k] = m->key[s];
      m2.val[k] = m->val[s];
    }
  pm_free(m);
  *m = m2;
  return 0;
}
static inline int32_t pm_find(const PtrMap* m, uintptr_t k) {
  size_t i = pm_slot(m, k);
  return m->key[i] ? m->val[i] : -1;
}

static PyObject *s_deps, *s_prefix, *s_group, *s_wants, *s_rootish, *s_wr, *s_hr, *s_rr;

static int names(void) {
  if (s_deps) return 0;
  s_deps = PyUnicode_InternFromString("dependencies");
  s_prefix = PyUnicode_InternFromString("prefix");
  s_group = PyUnicode_InternFromString("group");
  s_wants = PyUnicode_InternFromString("who_wants");
  s_rootish = PyUnicode_InternFromString("_rootish");
  s_wr = PyUnicode_InternFromString("worker_restrictions");
  s_hr = PyUnicode_InternFromString("host_restrictions");
  s_rr = PyUnicode_InternFromString("resource_restrictions");
  return s_deps && s_prefix && s_group && s_wants && s_rootish && s_wr && s_hr && s_rr ? 0 : -1;
}

// truth of attribute a of o (-1: error)
static int attr_true(PyObject* o, PyObject* a) {
  PyObject* v = PyObject_GetAttr(o, a);
  if (!v) return -1;
  int r = PyObject_IsTrue(v);
  Py_DECREF(v);
  return r;
}

// tasks: a list of TaskStates (the engine order). Outputs (caller-allocated, n entries
// unless stated): dep_count; dep_idx[cap] (rows in list order, each ascending: a position
// in the list, or -1 - m for misses[m]; graph_from_tasks re-sorts rows with misses);
// prefix_id / group_id; prefix_first /
// group_first (first task of each id, n entries reserved); n_ids[2] = #prefixes, #groups;
// wanted; rootish; restricted. misses: a list the outside dependencies are appended to.
// Returns the number of edges (> cap: nothing past cap was written; call again with room),
// or -1 with a Python exception set.
int64_t dgp_ingest_columns(PyObject* tasks, PyObject* misses, int64_t* dep_count, int64_t* dep_idx, int64_t cap,
                           int32_t* prefix_id, int32_t* group_id, int32_t* prefix_first, int32_t* group_first,
                           int32_t* n_ids, uint8_t* wanted, int8_t* rootish, uint8_t* restricted) {
  if (names()) return -1;
  if (!PyList_Check(tasks) || !PyList_Check(misses)) {
    PyErr_SetString(PyExc_TypeError, "dgp_ingest_columns: tasks and misses must be lists");
    return -1;
  }
  const Py_ssize_t n = PyList_Size(tasks);
  PtrMap tm, pm, gm, mm;
  memset(&tm, 0, sizeof tm);
  memset(&pm, 0, sizeof pm);
  memset(&gm, 0, sizeof gm);
  memset(&mm, 0, sizeof mm);
  int64_t ret = -1;
  if (pm_init(&tm, (size_t)n) || pm_init(&pm, 64) || pm_init(&gm, 1024) || pm_init(&mm, 64)) {
    PyErr_NoMemory();
    goto out;
  }
  int isnew;
  for (Py_ssize_t i = 0; i < n; i++) {  // list positions first: a row may name a later task
    PyObject* ts = PyList_GetItem(tasks, i);  // borrowed
    pm_get_or_add(&tm, (uintptr_t)ts, (int32_t)i, &isnew);
    if (!isnew) {
      PyErr_SetString(PyExc_ValueError, "dgp_ingest_columns: a task is listed twice");
      goto out;
    }
  }
  int32_t np_ = 0, ng = 0, nm = 0;
  int64_t e = 0;
  for (Py_ssize_t i = 0; i < n; i++) {
    PyObject* ts = PyList_GetItem(tasks, i);
    PyObject* deps = PyObject_GetAttr(ts, s_deps);
    if (!deps) goto out;
    PyObject* it = PyObject_GetIter(deps);
    Py_DECREF(deps);
    if (!it) goto out;
    int64_t c = 0;
    PyObject* d;
    while ((d = PyIter_Next(it))) {
      int32_t j = pm_find(&tm, (uintptr_t)d);
      if (j < 0) {  // an earlier graph's task: one misses entry per distinct object
        if (pm_reserve(&mm, (size_t)nm + 1)) {
          Py_DECREF(d);
          Py_DECREF(it);
          PyErr_NoMemory();
          goto out;
        }
        int32_t m = pm_get_or_add(&mm, (uintptr_t)d, nm, &isnew);
        if (isnew) {
          if (PyList_Append(misses, d)) {
            Py_DECREF(d);
            Py_DECREF(it);
            goto out;
          }
          nm++;
        }
        j = -1 - m;
      }
      Py_DECREF(d);
      if (e < cap) dep_idx[e] = j;
      e++;
      c++;
    }
    Py_DECREF(it);
    if (PyErr_Occurred()) goto out;
    dep_count[i] = c;
    if (e <= cap)  // the row ascending (insertion sort: rows are short)
      for (int64_t a = e - c + 1; a < e; a++) {
        const int64_t v = dep_idx[a];
        int64_t b = a - 1;
        while (b >= e - c && dep_idx[b] > v) {
          dep_idx[b + 1] = dep_idx[b];
          b--;
        }
        dep_idx[b + 1] = v;
      }
    // prefix / group ids, first seen
    PyObject* pf = PyObject_GetAttr(ts, s_prefix);
    if (!pf) goto out;
    if (pm_reserve(&pm, (size_t)np_ + 1)) {
      Py_DECREF(pf);
      PyErr_NoMemory();
      goto out;
    }
    int32_t q = pm_get_or_add(&pm, (uintptr_t)pf, np_, &isnew);
    Py_DECREF(pf);  // the TaskPrefix stays alive in SchedulerState.task_prefixes
    if (isnew) prefix_first[np_++] = (int32_t)i;
    prefix_id[i] = q;
    PyObject* gr = PyObject_GetAttr(ts, s_group);
    if (!gr) goto out;
    if (pm_reserve(&gm, (size_t)ng + 1)) {
      Py_DECREF(gr);
      PyErr_NoMemory();
      goto out;
    }
    int32_t h = pm_get_or_add(&gm, (uintptr_t)gr, ng, &isnew);
    Py_DECREF(gr);
    if (isnew) group_first[ng++] = (int32_t)i;
    group_id[i] = h;
    int w = attr_true(ts, s_wants);
    if (w < 0) goto out;
    wanted[i] = (uint8_t)w;
    PyObject* ro = PyObject_GetAttr(ts, s_rootish);
    if (!ro) goto out;
    if (ro == Py_None) {
      rootish[i] = -1;
    } else {
      int t = PyObject_IsTrue(ro);
      if (t < 0) {
        Py_DECREF(ro);
        goto out;
      }
      rootish[i] = (int8_t)t;
    }
    Py_DECREF(ro);
    int a = attr_true(ts, s_wr), b = a < 0 ? -1 : attr_true(ts, s_hr), r = b < 0 ? -1 : attr_true(ts, s_rr);
    if (r < 0) goto out;
    restricted[i] = (uint8_t)(a | (b << 1) | (r << 2));
  }
  n_ids[0] = np_;
  n_ids[1] = ng;
  ret = e;
out:
  pm_free(&tm);
  pm_free(&pm);
  pm_free(&gm);
  pm_free(&mm);
  return ret;
}
