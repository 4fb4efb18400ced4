"""MI355X-native batched NMPC solve step (drop-in for the ``ca.nlpsol`` call of
devsonni/MPC-Implementation ``Python/NMPC_TT.py``)."""
from .spec import ProblemSpec, Obstacle, make_spec, config_spec, LAYOUTS  # noqa: F401
from .nlpsol import nlpsol, Solver, RETURN_STATUS  # noqa: F401
from .scenarios import draw_scenarios, REFERENCE_OPTS  # noqa: F401
