"""Normalizer contract of the offline dataset (milo/milo/datasets.py:6-49) and the on-disk
trajectory databases the offline/expert sets are read from (milo/milo/utils.py:222-305)."""
from __future__ import annotations

import torch


def get_transformations(states: torch.Tensor, actions: torch.Tensor, next_states: torch.Tensor):
    """AmpDataset.get_transformations (datasets.py:23-43): (mu_s, sd_s, mu_a, sd_a, mu_d, sd_d)
    with sd = mean(|x - mu|) + 1e-8 (mean absolute deviation, not the std), Δ = s' - s."""
    diff = next_states - states
    state_mean = states.mean(dim=0).float()
    action_mean = actions.mean(dim=0).float()
    diff_mean = diff.mean(dim=0).float()
    state_scale = torch.abs(states - state_mean).mean(dim=0).float() + 1e-8
    action_scale = torch.abs(actions - action_mean).mean(dim=0).float() + 1e-8
    diff_scale = torch.abs(diff - diff_mean).mean(dim=0).float() + 1e-8
    return state_mean, state_scale, action_mean, action_scale, diff_mean, diff_scale


class AmpDataset(torch.utils.data.Dataset):
    """(s, a, s') triples (datasets.py:6-49)."""

    def __init__(self, states, actions, next_states, device=torch.device("cpu")):
        self.device = device
        self.states, self.actions, self.next_states = states, actions, next_states

    def get_transformations(self, device=None):
        dev = self.device if device is None else device
        return tuple(x.to(dev) for x in get_transformations(self.states, self.actions, self.next_states))

    def __len__(self):
        return self.states.size(0)

    def __getitem__(self, idx):
        return self.states[idx].float(), self.actions[idx].float(), self.next_states[idx].float()


# ---- on-disk trajectory databases (milo/milo/utils.py:222-305) ----------------------------
# The reference's collect_data.py / collect_expert.py torch.save a list of per-trajectory
# dicts: offline {'episode': (states [T+1,S], actions [T,A], rewards), 'dtw_cost' | 'ep_rew'},
# expert {'episode': states [T+1,S]}.  They hold numpy arrays, so they are read with the
# weights-only unpickler plus an allow-list of numpy's array/scalar reconstructors only
# (nothing in the file can name any other callable).


def _numpy_safe_globals():
    import numpy as np
    try:
        from numpy._core import multiarray as ma
    except ImportError:  # numpy < 2
        from numpy.core import multiarray as ma
    allowed = [ma._reconstruct, ma.scalar, np.ndarray, np.dtype,
               (ma._reconstruct, "numpy.core.multiarray._reconstruct"),  # pickles written by numpy 1.x
               (ma.scalar, "numpy.core.multiarray.scalar")]
    dtypes = getattr(np, "dtypes", None)  # numpy >= 1.25 pickles dtypes by their class
    if dtypes is not None:
        for n in ("Float16DType", "Float32DType", "Float64DType", "Int8DType", "Int16DType", "Int32DType",
                  "Int64DType", "UInt8DType", "UInt16DType", "UInt32DType", "UInt64DType", "BoolDType"):
            if hasattr(dtypes, n):
                allowed.append(getattr(dtypes, n))
    return allowed


def load_db(db_path):
    """torch.load of a trajectory database with the weights-only unpickler (numpy arrays and
    scalars allowed, nothing else)."""
    with torch.serialization.safe_globals(_numpy_safe_globals()):
        return torch.load(db_path, map_location="cpu", weights_only=True)


def _select(saved_db, num_trajs, idx):
    if isinstance(num_trajs, str) and num_trajs == "all":  # the reference tests `is 'all'`
        num_trajs = len(saved_db)
    saved_db = saved_db[:num_trajs]
    if idx is not None:
        # utils.py:253 indexes the list and then iterates the single dict it got (its keys);
        # get_paths_mjrl (:295) wraps it in a list, which is what both do here
        saved_db = [saved_db[idx]]
    return saved_db, num_trajs


def get_db_mjrl(db_path, num_trajs="all", idx=None, expert=False, imitate_amp=True, verbose=True):
    """utils.py:244-282: the database as float32 tensors (s, a, s') — expert: (s, s') — with
    s = episode states[:-1], s' = states[1:], trajectories concatenated in file order."""
    import numpy as np
    saved_db, num_trajs = _select(load_db(db_path) if isinstance(db_path, (str, bytes)) or hasattr(db_path, "read")
                                  else db_path, num_trajs, idx)
    states, actions, next_states, total_reward = [], [], [], 0
    mean_db_reward = None
    for traj in saved_db:
        if expert:
            all_state = traj["episode"]
            states.append(all_state[:-1])
            next_states.append(all_state[1:])
        else:
            all_state, action, _ = traj["episode"]
            states.append(all_state[:-1])
            actions.append(action)
            next_states.append(all_state[1:])
            total_reward += traj["dtw_cost"] if imitate_amp else traj["ep_rew"]
            mean_db_reward = total_reward / num_trajs
    if expert:
        return (torch.from_numpy(np.concatenate(states, axis=0)).float(),
                torch.from_numpy(np.concatenate(next_states, axis=0)).float())
    db = (torch.from_numpy(np.concatenate(states, axis=0)).float(),
          torch.from_numpy(np.concatenate(actions, axis=0)).float(),
          torch.from_numpy(np.concatenate(next_states, axis=0)).float())
    if verbose:
        print(f"{'DB DTW Cost' if imitate_amp else 'DB Mean Reward'}: {mean_db_reward} | DB # Samples: {db[0].shape[0]}")
    return db


def get_paths_mjrl(db_path, num_trajs="all", idx=None, expert=False):
    """utils.py:288-305: mjrl-style paths ({'observations', 'actions'}; expert
    {'observations', 'next_observation'}) for behaviour-cloning warm starts."""
    saved_db, _ = _select(load_db(db_path) if isinstance(db_path, (str, bytes)) or hasattr(db_path, "read")
                          else db_path, num_trajs, idx)
    paths = []
    for traj in saved_db:
        if expert:
            all_state = traj["episode"]
            paths.append({"observations": all_state[:-1], "next_observation": all_state[1:]})
        else:
            all_state, action, _ = traj["episode"]
            paths.append({"observations": all_state[:-1], "actions": action})
    return paths


def convert_to_veltopos(path, deepmimic=None, is_db_mjrl=False, is_expert=False, vel_offset=None, dt=None):
    """utils.py:222-241: scale the velocity block (columns >= vel_offset) by dt = 1/update
    rate, in place on the loaded object, which is returned.  `deepmimic` supplies
    get_vel_offset()/get_agent_update_rate() as in the reference; or pass vel_offset and dt.
    The db-format expert branch scales the single column vel_offset of x[1], as the
    reference does (utils.py:229, `x[1][:, vel_offset]`)."""
    x = load_db(path) if isinstance(path, (str, bytes)) or hasattr(path, "read") else path
    if deepmimic is not None:
        vel_offset = deepmimic.get_vel_offset()
        dt = 1 / deepmimic.get_agent_update_rate()
    if is_db_mjrl:
        x[0][:, vel_offset:] *= dt
        if is_expert:
            x[1][:, vel_offset] *= dt
        else:
            x[2][:, vel_offset:] *= dt
    else:
        for i in x:
            if is_expert:
                i["episode"][:, vel_offset:] *= dt
            else:
                i["episode"][0][:, vel_offset:] *= dt
    return x
