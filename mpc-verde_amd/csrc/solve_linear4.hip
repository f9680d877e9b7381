// solve_linear4.hip -- solve/plant/shift/constraint kernels of LinearModel<4, 1>: Trajectory_tracking_dynamic_model.py:117-145 (config 4).
#include "kernels.h"

namespace mpcx {
using Linear4x1 = LinearModel<4, 1>;
}
MPCX_INSTANTIATE(Linear4x1, linear4, "mpcx::LinearModel<4, 1>")
