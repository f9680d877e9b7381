// solve_linear4x2.hip -- solve/plant/shift/constraint kernels of LinearModel<4, 2>: two-input linear
// models (nx <= 4 through the host-side zero-state embedding, mpcx/lti.py StatePad), e.g. a unicycle
// linearised about a reference (x, y, th; v, w) -- the LTV form of Casadi/multiple_shooting_casadi.py:68-72.
#include "kernels.h"

namespace mpcx {
using Linear4x2 = LinearModel<4, 2>;
}
MPCX_INSTANTIATE(Linear4x2, linear4x2, "mpcx::LinearModel<4, 2>")
