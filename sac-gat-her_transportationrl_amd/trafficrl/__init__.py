"""trafficrl -- MI355X-native vectorised traffic-repair env (hot path of
pop-pop-pOp-dev/SAC-GAT-HER_transportationRL) on gfx950 HIP kernels.

Module layout mirrors the reference's src/ tree:
  trafficrl.data.tntp_parser   <- src/data/tntp_parser.py
  trafficrl.env.repair_env     <- src/env/repair_env.py  (RepairEnv facade)
  trafficrl.env.vec_env        (batched VecRepairEnv, the performance path)
  trafficrl.baselines          <- src/baselines/__init__.py
  trafficrl.models / rl / train <- src/models, src/rl, src/train.py
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
