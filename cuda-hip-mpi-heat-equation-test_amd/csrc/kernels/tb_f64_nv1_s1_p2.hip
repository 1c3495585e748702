// Instantiation unit: temporal-blocked stencil, double, 1 x 16 B per lane,
// skew-1 level pipeline, 6-row prefetch, K = 1..16.
#include "tb_impl.hpp"

namespace heat2d {
namespace kern {
namespace tbimpl {

template <>
void dispatch<double, 1, 1, 2>(int k, unsigned nblocks, const double* src, double* dst, const TbArgs& a, double r,
                                 hipStream_t s) {
  switch (k) {
    H2D_TB_CASE(double, 1, 1, 2, 1)
    H2D_TB_CASE(double, 1, 1, 2, 2)
    H2D_TB_CASE(double, 1, 1, 2, 3)
    H2D_TB_CASE(double, 1, 1, 2, 4)
    H2D_TB_CASE(double, 1, 1, 2, 5)
    H2D_TB_CASE(double, 1, 1, 2, 6)
    H2D_TB_CASE(double, 1, 1, 2, 7)
    H2D_TB_CASE(double, 1, 1, 2, 8)
    H2D_TB_CASE(double, 1, 1, 2, 9)
    H2D_TB_CASE(double, 1, 1, 2, 10)
    H2D_TB_CASE(double, 1, 1, 2, 11)
    H2D_TB_CASE(double, 1, 1, 2, 12)
    H2D_TB_CASE(double, 1, 1, 2, 13)
    H2D_TB_CASE(double, 1, 1, 2, 14)
    H2D_TB_CASE(double, 1, 1, 2, 15)
    H2D_TB_CASE(double, 1, 1, 2, 16)
    default:
      break;
  }
  HEAT2D_REQUIRE(false, "temporal depth not instantiated for this variant");
}

template <>
int occupancy_blocks<double, 1, 1, 2>(int k) {
  switch (k) {
    H2D_OCC_CASE(double, 1, 1, 2, 1)
    H2D_OCC_CASE(double, 1, 1, 2, 2)
    H2D_OCC_CASE(double, 1, 1, 2, 3)
    H2D_OCC_CASE(double, 1, 1, 2, 4)
    H2D_OCC_CASE(double, 1, 1, 2, 5)
    H2D_OCC_CASE(double, 1, 1, 2, 6)
    H2D_OCC_CASE(double, 1, 1, 2, 7)
    H2D_OCC_CASE(double, 1, 1, 2, 8)
    H2D_OCC_CASE(double, 1, 1, 2, 9)
    H2D_OCC_CASE(double, 1, 1, 2, 10)
    H2D_OCC_CASE(double, 1, 1, 2, 11)
    H2D_OCC_CASE(double, 1, 1, 2, 12)
    H2D_OCC_CASE(double, 1, 1, 2, 13)
    H2D_OCC_CASE(double, 1, 1, 2, 14)
    H2D_OCC_CASE(double, 1, 1, 2, 15)
    H2D_OCC_CASE(double, 1, 1, 2, 16)
    default:
      break;
  }
  return 1;
}

}  // namespace tbimpl
}  // namespace kern
}  // namespace heat2d
