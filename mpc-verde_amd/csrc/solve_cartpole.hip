// solve_cartpole.hip -- solve/plant/shift/constraint kernels of OdeModel<CartPole>: BASELINE config 5 (cart-pole swing-up).
#include "kernels.h"

MPCX_INSTANTIATE(OdeModel<CartPole>, cartpole, "mpcx::OdeModel<mpcx::CartPole>")
