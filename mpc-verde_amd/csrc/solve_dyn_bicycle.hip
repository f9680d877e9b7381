// solve_dyn_bicycle.hip -- solve/plant/shift/constraint kernels of OdeModel<DynBicycle>: BASELINE config 4 (6-state dynamic bicycle).
#include "kernels.h"

MPCX_INSTANTIATE(OdeModel<DynBicycle>, dyn_bicycle, "mpcx::OdeModel<mpcx::DynBicycle>")
