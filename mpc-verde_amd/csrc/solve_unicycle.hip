// solve_unicycle.hip -- solve/plant/shift/constraint kernels of UnicycleModel: Casadi/multiple_shooting_casadi.py:68-114 (configs 1-3).
#include "kernels.h"

MPCX_INSTANTIATE(UnicycleModel, unicycle, "mpcx::UnicycleModel")
