// Instantiation unit: persistent multi-cycle temporal-blocked stencil (float, ring 4,
// arithmetic AR = 1; one co-resident wave per item, neighbour-counter sync between
// cycles — see tb_impl.hpp tb_persist_kernel).
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {
H2D_PS_UNIT(float, 4, 1, H2D_TB_CASES_F32DEEP)
}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
