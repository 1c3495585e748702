// Instantiation unit: wave-pair kernel (tb_pair_kernel), float, ring of 4 level-0 rows,
// arith 0 (0 reference rounding, 1 fma, 2 r = 1/4), K = 2..16 (see tb_impl.hpp).
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {
H2D_PR_UNIT(4, 0)
}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
