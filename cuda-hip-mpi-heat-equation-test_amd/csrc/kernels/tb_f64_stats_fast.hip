// Instantiation unit: temporal-blocked stencil with fused statistics of the stored level
// (double, ring 4, general kernel, scaled-level arithmetic AR = 3 (any r); see tb_impl.hpp StatAcc).
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {
H2D_ST_UNIT(double, 3, H2D_TB_CASES_DEEP)
}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
