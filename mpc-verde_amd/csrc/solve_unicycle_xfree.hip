// solve_unicycle_xfree.hip -- kernels of UnicycleFreeModel: the unicycle without state bounds (configs 1-2, Casadi/multiple_shooting_casadi.py:42-45).
#include "kernels.h"

MPCX_INSTANTIATE(UnicycleFreeModel, unicycle_xfree, "mpcx::UnicycleFreeModel")
