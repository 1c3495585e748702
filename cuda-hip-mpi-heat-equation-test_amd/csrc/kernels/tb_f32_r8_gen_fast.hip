// Instantiation unit: temporal-blocked stencil, float, 16 B per lane, ring of 8 level-0 rows (6 in
// flight), general kernel, arith 3 (fast), K = 1..16 — single launches of small grids (see tb_impl.hpp).
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {
H2D_TB_UNIT(float, 8, false, 3)
}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
