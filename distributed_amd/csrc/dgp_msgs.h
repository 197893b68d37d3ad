// compute-task message fields of a batch of placements, from the resident state
// (SchedulerState._task_to_msg, scheduler.py:3421-3450).
//
// For placements [offset, offset + count) of the placement log: every dependency of the
// placed task (CSR order of the graph), its TaskState.nbytes as _task_to_msg sends it (raw,
// -1 when none was reported) and its who_has now (ascending worker index: holder_of, or the
// bitset row once replicas were added, TD_MULTI). One thread per placement; two passes (the
// counts, then the rows at the host-scanned offsets). Read right after the engine call that
// made the placements, as _add_to_processing builds the message before any later stimulus.
#pragma once

namespace dgp {
namespace msg {

__device__ __forceinline__ bool multi_row(const Dev& D, int d) { return (D.evf & EVF_MULTI) && (D.tdyn[d] & TD_MULTI); }

__device__ __forceinline__ int who_has_count(const Dev& D, int d) {
  if (multi_row(D, d)) {
    int n = 0;
    for (int b = 0; b < D.WB; b++) n += __builtin_popcountll(D.holders[(size_t)d * D.WB + b]);
    return n;
  }
  return D.holder_of[d] >= 0 ? 1 : 0;
}

// per placement: dependencies, holders over all of them
__global__ void __launch_bounds__(256) k_msg_count(const Dev* __restrict__ Dp, long long offset, int count,
                                                   int32_t* __restrict__ ndep, int32_t* __restrict__ nhold) {
  const Dev& D = *Dp;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  const int t = D.pl_task[offset + j];
  int nd = 0, nh = 0;
  if (t >= 0 && t < D.N) {
    for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++) {
      nh += who_has_count(D, D.dep_idx[k]);
      nd++;
    }
  }
  ndep[j] = nd;
  nhold[j] = nh;
}

// per placement: its rows at dep_ptr[j] / hold_base[j] (exclusive scans of the counts)
__global__ void __launch_bounds__(256) k_msg_fill(const Dev* __restrict__ Dp, long long offset, int count,
                                                  const int64_t* __restrict__ dep_ptr,
                                                  const int64_t* __restrict__ hold_base,
                                                  int32_t* __restrict__ dep_task, int64_t* __restrict__ dep_nbytes,
                                                  int32_t* __restrict__ dep_hcount, int32_t* __restrict__ holder_idx) {
  const Dev& D = *Dp;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  const int t = D.pl_task[offset + j];
  if (t < 0 || t >= D.N) return;
  int64_t pos = dep_ptr[j], hp = hold_base[j];
  for (int64_t k = D.dep_ptr[t]; k < D.dep_ptr[t + 1]; k++, pos++) {
    const int d = D.dep_idx[k];
    dep_task[pos] = d;
    dep_nbytes[pos] = D.cur_nbytes[d];
    int n = 0;
    if (multi_row(D, d)) {
      for (int b = 0; b < D.WB; b++) {
        for (unsigned long long m = D.holders[(size_t)d * D.WB + b]; m; m &= m - 1) {
          holder_idx[hp + n] = b * 64 + __builtin_ctzll(m);
          n++;
        }
      }
    } else if (D.holder_of[d] >= 0) {
      holder_idx[hp] = D.holder_of[d];
      n = 1;
    }
    dep_hcount[pos] = n;
    hp += n;
  }
}

}  // namespace msg
}  // namespace dgp
