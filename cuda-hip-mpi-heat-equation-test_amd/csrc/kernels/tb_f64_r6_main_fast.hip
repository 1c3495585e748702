// Instantiation unit (scaled-level arithmetic for any r, AR = 3): temporal-blocked stencil, double, 16 B per lane, ring of
// 6 level-0 rows, interior-only (MAIN) kernel, K = 1..24 (see tb_impl.hpp).
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {
H2D_TB_UNIT_F64(double, 6, true, 3)
}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
