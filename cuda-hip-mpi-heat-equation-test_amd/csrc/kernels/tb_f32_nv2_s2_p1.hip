// Instantiation unit: temporal-blocked stencil, float, 2 x 16 B per lane,
// skew-2 level pipeline, 3-row prefetch, K = 1..8.
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {

template <>
void dispatch<float, 2, 2, 1>(int k, unsigned nblocks, const float* src, float* dst, const TbArgs& a, float r,
                                 hipStream_t s) {
  switch (k) {
    H2D_TB_CASE(float, 2, 2, 1, 1)
    H2D_TB_CASE(float, 2, 2, 1, 2)
    H2D_TB_CASE(float, 2, 2, 1, 3)
    H2D_TB_CASE(float, 2, 2, 1, 4)
    H2D_TB_CASE(float, 2, 2, 1, 5)
    H2D_TB_CASE(float, 2, 2, 1, 6)
    H2D_TB_CASE(float, 2, 2, 1, 7)
    H2D_TB_CASE(float, 2, 2, 1, 8)
    default:
      break;
  }
  HEAT2D_REQUIRE(false, "temporal depth not instantiated for this variant");
}

template <>
int occupancy_blocks<float, 2, 2, 1>(int k) {
  switch (k) {
    H2D_OCC_CASE(float, 2, 2, 1, 1)
    H2D_OCC_CASE(float, 2, 2, 1, 2)
    H2D_OCC_CASE(float, 2, 2, 1, 3)
    H2D_OCC_CASE(float, 2, 2, 1, 4)
    H2D_OCC_CASE(float, 2, 2, 1, 5)
    H2D_OCC_CASE(float, 2, 2, 1, 6)
    H2D_OCC_CASE(float, 2, 2, 1, 7)
    H2D_OCC_CASE(float, 2, 2, 1, 8)
    default:
      break;
  }
  return 1;
}

}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
