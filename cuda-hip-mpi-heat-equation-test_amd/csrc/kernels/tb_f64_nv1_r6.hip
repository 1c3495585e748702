// Instantiation unit: temporal-blocked stencil, double, 1 x 16 B per lane,
// ring of 6 level-0 rows, K = 1..16 (see tb_impl.hpp).
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {
H2D_TB_UNIT(double, 1, 6)
}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
