// nslam_query_dec.hip — one decoder's backward kernels (k_dec_bwd instantiations + launchers),
// compiled once per decoder with -DNSLAM_DEC=<NSLAM_DEC_*> (Makefile) so the library's heaviest
// templates build in parallel.
#ifndef NSLAM_DEC
#error "build with -DNSLAM_DEC=0..3"
#endif
#include "nslam_query_impl.h"

namespace nslamq {
template int dispatch_dec_bwd<NSLAM_DEC>(const QueryKArgs&, bool, float*, hipStream_t);
}  // namespace nslamq
