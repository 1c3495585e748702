// Instantiation unit: interior kernel of the fused cycle (float, ring 4, arithmetic
// AR = 0; device-scope row stores, band items counted for the gated exchange —
// tb_impl.hpp kVarFused, stencil_tb.hip plan_fused).
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {
H2D_FU_UNIT(float, 4, 0, H2D_TB_CASES_F32DEEP)
}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
