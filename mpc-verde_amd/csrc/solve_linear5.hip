// solve_linear5.hip -- solve/plant/shift/constraint kernels of LinearModel<5, 1>: inverted_pendulum_single_shooting_mpctools.py:15-64 (config 5).
#include "kernels.h"

namespace mpcx {
using Linear5x1 = LinearModel<5, 1>;
}
MPCX_INSTANTIATE(Linear5x1, linear5, "mpcx::LinearModel<5, 1>")
