// sbr_multi.h — internal interface of the multi-GPU fan-out (sbr_multi.hip) used by
// the C-ABI entry points of sbr_capi.hip.  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

#include "../../include/sbr.h"
#include "sbr_shard.h"

struct sbr_multi;

// the private stream of a single-device context (sbr_capi.hip): a rank's sweeps run on it
hipStream_t sbr_ctx_stream(sbr_ctx* c);

namespace sbr_multi_impl {

using FieldSpec = sbr_shard::Field;

// stage(rank, n_cols_of_rank, device_in, stream): copy the rank's inputs into device_in
using StageFn = std::function<int(int, int64_t, void*, hipStream_t)>;
// run(rank, n_cols_of_rank, child_ctx, stream, device_in, device_field_ptrs): enqueue the sweep
using RunFn = std::function<int(int, int64_t, sbr_ctx*, hipStream_t, void*, const std::vector<void*>&)>;

int create(int n_gpus, const int* devices, sbr_multi** out, std::vector<sbr_ctx*>& kids, std::string& err);
void destroy(sbr_multi* m);
int size(const sbr_multi* m);
sbr_ctx* child(sbr_multi* m, int rank);
const char* last_error(const sbr_multi* m);
// phases of the last sweep, ms (sbr_host_phases on an n-device context)
const double* phases(const sbr_multi* m);
// rccl_gather: results to rank 0 over RCCL, then scattered from there (SBR_FLAG_RCCL_GATHER);
// otherwise every rank copies its own columns into the caller's arrays
int run_sharded(sbr_multi* m, int64_t n_col, int64_t n_u, const std::vector<FieldSpec>& fields, size_t in_bytes,
                const StageFn& stage, const RunFn& run, bool rccl_gather = false);

}  // namespace sbr_multi_impl
