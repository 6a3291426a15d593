// Token GEMM instantiations for a 48-deep K stage (see gemm_tok.h).
#include "gemm_tok.h"

namespace msu_tok {
int dispatch_k48(int dtype, const TokPlan& p, const TokArgs& a, int epi, bool bias, bool concat, hipStream_t st) {
  if (dtype == MSU_F16) return dispatch_nc<f16_t, 48, false>(p, a, epi, bias, concat, st);
  return dispatch_nc<bf16_t, 48, false>(p, a, epi, bias, concat, st);
}
}  // namespace msu_tok
