// solve_kin_bicycle.hip -- solve/plant/shift/constraint kernels of OdeModel<KinBicycle>: BASELINE config 3 (kinematic bicycle).
#include "kernels.h"

MPCX_INSTANTIATE(OdeModel<KinBicycle>, kin_bicycle, "mpcx::OdeModel<mpcx::KinBicycle>")
