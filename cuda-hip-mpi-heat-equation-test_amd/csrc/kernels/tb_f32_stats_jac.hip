// Instantiation unit: temporal-blocked stencil with fused statistics of the stored level
// (float, ring 4, general kernel, r = 1/4 arithmetic AR = 2; see tb_impl.hpp StatAcc).
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {
H2D_ST_UNIT(float, 2, H2D_TB_CASES_F32DEEP)
}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
