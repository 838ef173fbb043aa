"""mppi_hip — MI355X-native MPPI solve engine (libmppi_hip.so) with the reference controller API.

    from mppi_hip import MPPIModel, mppi_controller, SimData
    model = MPPIModel("cartpole_py")            # src/cartpole_mppi.py constants, analytic cartpole dynamics
    mppi_controller(model, data)                # data.ctrl <- U[:,0], U_global shifted

The package directory is humanoid_mppi-rl_amd/ (not importable by name); put it on sys.path, e.g.
sys.path.insert(0, "<repo>/humanoid_mppi-rl_amd").
"""
from . import _lib
from ._lib import MPPIError, MPPILibraryError
from .controller import (MPPIModel, SimData, mppi_controller, mppi_step, mppi_update, rollout,
                         rollout_learned_model_batched)
from .engine import Config, Engine, SolveResult
from .nets import (cross_attention_blob, feature_attention_blob, load_npz, mlp_blob, pack_blob,
                   synthetic_feature_attention, synthetic_mlp)

__all__ = ["Config", "Engine", "SolveResult", "MPPIModel", "SimData", "rollout", "mppi_step", "mppi_controller",
           "mppi_update", "rollout_learned_model_batched", "MPPIError", "MPPILibraryError", "pack_blob", "load_npz",
           "cross_attention_blob", "feature_attention_blob", "mlp_blob", "synthetic_mlp", "synthetic_feature_attention"]
