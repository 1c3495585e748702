// Instantiation unit: temporal-blocked stencil, double, 1 x 16 B per lane,
// skew-1 level pipeline, 3-row prefetch, K = 1..16.
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {

template <>
void dispatch<double, 1, 1, 1>(int k, unsigned nblocks, const double* src, double* dst, const TbArgs& a, double r,
                                 hipStream_t s) {
  switch (k) {
    H2D_TB_CASE(double, 1, 1, 1, 1)
    H2D_TB_CASE(double, 1, 1, 1, 2)
    H2D_TB_CASE(double, 1, 1, 1, 3)
    H2D_TB_CASE(double, 1, 1, 1, 4)
    H2D_TB_CASE(double, 1, 1, 1, 5)
    H2D_TB_CASE(double, 1, 1, 1, 6)
    H2D_TB_CASE(double, 1, 1, 1, 7)
    H2D_TB_CASE(double, 1, 1, 1, 8)
    H2D_TB_CASE(double, 1, 1, 1, 9)
    H2D_TB_CASE(double, 1, 1, 1, 10)
    H2D_TB_CASE(double, 1, 1, 1, 11)
    H2D_TB_CASE(double, 1, 1, 1, 12)
    H2D_TB_CASE(double, 1, 1, 1, 13)
    H2D_TB_CASE(double, 1, 1, 1, 14)
    H2D_TB_CASE(double, 1, 1, 1, 15)
    H2D_TB_CASE(double, 1, 1, 1, 16)
    default:
      break;
  }
  HEAT2D_REQUIRE(false, "temporal depth not instantiated for this variant");
}

template <>
int occupancy_blocks<double, 1, 1, 1>(int k) {
  switch (k) {
    H2D_OCC_CASE(double, 1, 1, 1, 1)
    H2D_OCC_CASE(double, 1, 1, 1, 2)
    H2D_OCC_CASE(double, 1, 1, 1, 3)
    H2D_OCC_CASE(double, 1, 1, 1, 4)
    H2D_OCC_CASE(double, 1, 1, 1, 5)
    H2D_OCC_CASE(double, 1, 1, 1, 6)
    H2D_OCC_CASE(double, 1, 1, 1, 7)
    H2D_OCC_CASE(double, 1, 1, 1, 8)
    H2D_OCC_CASE(double, 1, 1, 1, 9)
    H2D_OCC_CASE(double, 1, 1, 1, 10)
    H2D_OCC_CASE(double, 1, 1, 1, 11)
    H2D_OCC_CASE(double, 1, 1, 1, 12)
    H2D_OCC_CASE(double, 1, 1, 1, 13)
    H2D_OCC_CASE(double, 1, 1, 1, 14)
    H2D_OCC_CASE(double, 1, 1, 1, 15)
    H2D_OCC_CASE(double, 1, 1, 1, 16)
    default:
      break;
  }
  return 1;
}

}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
