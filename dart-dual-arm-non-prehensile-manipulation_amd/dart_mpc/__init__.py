"""dart_mpc -- MI355X-native batched tray-tilt NMPC solver for DART.

Drop-in for the reference's MPC hot path:
  - ``PMPC``            <- PMPC/src/controller/mpc_3d.py:11-138
  - ``mpc_worker``      <- PMPC/main_parallel_enhanced.py:22-55
  - ``mpc_batch_server`` <- the per-simulation worker fan-out of main_parallel_enhanced.py:200-207,
                            as one process batching every simulation's queue
  - ``AdaptiveNPMPCSmooth``, ``RLS`` <- RMPC/dev_dual/controller/np_mpc_adaptive_with_linear_regressor.py
  - ``RMPCStep``        <- RMPC/dev_dual/rob_ctrl.py:331-352 (RLS fused into the solve launch)
  - ``RLMPC``, ``LmpcPolicy``, ``LmpcSolver`` <- LMPC/src/controller/rlmpc2.py (solver worker, policy worker, front-end)
  - ``RLMPCAsync``, ``lmpc_solver_worker``, ``lmpc_policy_worker`` <- the same with the reference's shared-memory /
                           Event process topology (rlmpc2.py:110-164, 229-533, 537-769, 986-1021)
  - ``ArmControl``, ``ArmSolver`` <- ARMCONTROL (PMPC/src/controller/arm.py), the per-arm impedance QP
  - ``harness``         <- the closed loops of main_parallel_enhanced.py / rob_ctrl.py without MuJoCo, and the
                           reference's result formats (logger.py npz + metrics, rob_ctrl.py episode JSON)
  - ``Solver``, ``RmpcSolver``  the C ABI of include/dart_mpc.h (libdartmpc.so)
"""
from ._lib import DartMPCError, LmpcSolver, RmpcSolver, Solver, build, lib, rls_update_batch, STATUS_NAMES  # noqa: F401
from .pmpc import PMPC, tilt_to_quat  # noqa: F401
from .worker import mpc_worker  # noqa: F401
from .batch_server import mpc_batch_server  # noqa: F401
from .rmpc import AdaptiveNPMPCSmooth, RLS, RMPCStep  # noqa: F401
from .lmpc import RLMPC, LmpcPolicy, init_policy_weights, policy_solve_batch  # noqa: F401
from .lmpc_shm import RLMPCAsync, lmpc_policy_worker, lmpc_solver_worker  # noqa: F401
from .arm import ArmControl, ArmSolver  # noqa: F401
from .mjdata import BodyData  # noqa: F401
from . import harness, workload  # noqa: F401

__all__ = ["PMPC", "mpc_worker", "mpc_batch_server", "Solver", "RmpcSolver", "LmpcSolver", "RLMPC", "LmpcPolicy", "init_policy_weights", "policy_solve_batch", "RLMPCAsync", "lmpc_solver_worker", "lmpc_policy_worker", "ArmControl", "ArmSolver", "AdaptiveNPMPCSmooth", "RLS", "RMPCStep", "DartMPCError",
           "build", "lib", "rls_update_batch", "tilt_to_quat", "workload", "harness", "BodyData"]
