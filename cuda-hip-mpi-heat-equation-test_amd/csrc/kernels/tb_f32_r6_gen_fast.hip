// Instantiation unit (scaled-level arithmetic for any r, AR = 3): temporal-blocked stencil, float, 16 B per lane, ring of
// 6 level-0 rows, general (edge-classifying) kernel, K = 1..16 (see tb_impl.hpp).
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {
H2D_TB_UNIT(float, 6, false, 3)
}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
