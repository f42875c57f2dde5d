"""amp_extensions_amd — MI355X-native learned-dynamics rollout path of amp_extensions.

The gym_simenv learned-dynamics step (4-model dense-MLP ensemble), the MILO RFF-MMD
cost with the ensemble-disagreement bonus, the AMP/GAIL least-squares discriminator
reward and the humanoid3d fall/horizon termination, as hand-written HIP kernels for
gfx950 behind a C ABI (include/amx_hip.h, libamx_hip.so) and the reference's Python
surfaces (SimEnv, sample_points, RBFLinearCost, GAILCost, DynamicsEnsemble), plus the
sampler's consumers: returns, MLP value baseline and GAE (mjrl process_samples) and the
NPG policy update (mjrl npg_cg).

The native library is loaded on first use; there is no CPU fallback.
"""
from .humanoid import TerminationConfig  # noqa: F401

__all__ = [
    "AmxContext", "DeviceEnsemble", "RffMap", "RolloutEngine", "RBFLinearCost", "GAILCost", "DevicePolicy",
    "TerminationConfig", "SimEnv", "BatchedSimEnv", "sample_points", "DeviceMLPBaseline", "process_samples",
    "DeviceNPG",
]


def __getattr__(name):
    if name in ("AmxContext", "DeviceEnsemble", "RffMap"):
        from . import engine
        return getattr(engine, name)
    if name in ("RBFLinearCost", "GAILCost"):
        from . import costs
        return getattr(costs, name)
    if name == "DevicePolicy":
        from .policy import DevicePolicy
        return DevicePolicy
    if name == "RolloutEngine":
        from .rollout import RolloutEngine
        return RolloutEngine
    if name in ("SimEnv", "BatchedSimEnv"):
        from . import sim_env
        return getattr(sim_env, name)
    if name in ("DeviceMLPBaseline", "process_samples"):
        from . import gae
        return getattr(gae, name)
    if name == "DeviceNPG":
        from .npg import DeviceNPG
        return DeviceNPG
    if name == "sample_points":
        from .sampler import sample_points
        return sample_points
    raise AttributeError(name)
