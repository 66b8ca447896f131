from .repair_env import EnvState, RepairEnv  # noqa: F401
from .vec_env import VecObs, VecRepairEnv  # noqa: F401
