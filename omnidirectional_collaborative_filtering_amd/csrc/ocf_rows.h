// The row-stream weight-gradient launches (ocf_rows.hip) as ocf_gemm.hip sees them.
#pragma once
#include "ocf_epilogues.h"
#include "ocf_optim_ws.h"

namespace ocf {
// tuning switches (ocf_set_tuning)
extern int g_optim_rows, g_rows_long, g_rows_small_waves, g_pair_wait_polls, g_rows_dual,
    g_rows_dual_count, g_rows_dual_parts, g_rows_dual_large, g_rows_dual_pf;
int cu_count();
WsJobs ws_jobs(const OcfGemmArgs& g);
// EPI_OPTIM through the row-stream kernel; false when the arguments need a tile kernel instead
template <typename CT>
bool launch_rows(const OcfGemmArgs& g, const EpiOptim::Params& ep, hipStream_t s);
// ocf_gemm_pair's one launch; false when the two updates cannot share it (then two launches)
template <typename CT>
bool launch_rows_pair(const OcfGemmArgs& a, const OcfGemmArgs& b, OcfPairSync& sync, hipStream_t s);
}  // namespace ocf
