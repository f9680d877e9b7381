"""mpcx -- MI355X-native batched multiple-shooting MPC (drop-in for the CasADi/IPOPT
hot path of gabrielhaj/mpc-verde).  See DESIGN.md and include/mpcx.h."""
from .ocp import OCP, unicycle_point_to_point, unicycle_point_to_point_mpctools, unicycle_tracking, to_spec  # noqa: F401,E501
from .nlpsol import Solver, Integrator, nlpsol, integrator  # noqa: F401
from .lti import LinearOCP, inverted_pendulum_qp, lateral_ltv, lateral_error_lti, c2d  # noqa: F401
from .ode import OdeOCP, kinematic_bicycle_tracking, dynamic_bicycle_lane_change, cartpole_swingup  # noqa: F401
from .record import ClosedLoopLog  # noqa: F401
from .nmpc import ControlSolver, nmpc, callSolver  # noqa: F401
from . import _lib  # noqa: F401

__all__ = ["OCP", "unicycle_point_to_point", "unicycle_point_to_point_mpctools", "unicycle_tracking", "to_spec", "Solver", "Integrator", "nlpsol",
           "integrator", "LinearOCP",
           "inverted_pendulum_qp", "lateral_ltv", "lateral_error_lti", "c2d", "ClosedLoopLog", "OdeOCP", "kinematic_bicycle_tracking",
           "dynamic_bicycle_lane_change", "cartpole_swingup", "ControlSolver", "nmpc", "callSolver"]
