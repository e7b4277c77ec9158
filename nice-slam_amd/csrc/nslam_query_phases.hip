// nslam_query_phases.hip — the whole query path in ONE translation unit (phase-timing build: the
// s_memtime buffer g_phase must be a single device symbol that nslam_debug_phases can read).
#define NSLAM_QUERY_ONE_TU
#include "nslam_query.hip"

namespace nslamq {
template int dispatch_dec_bwd<NSLAM_DEC_COARSE>(const QueryKArgs&, bool, float*, hipStream_t);
template int dispatch_dec_bwd<NSLAM_DEC_MIDDLE>(const QueryKArgs&, bool, float*, hipStream_t);
template int dispatch_dec_bwd<NSLAM_DEC_FINE>(const QueryKArgs&, bool, float*, hipStream_t);
template int dispatch_dec_bwd<NSLAM_DEC_COLOR>(const QueryKArgs&, bool, float*, hipStream_t);
}  // namespace nslamq

#include "nslam_query_multi.hip"
#include "nslam_color_wgrad.hip"
