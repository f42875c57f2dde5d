"""Normalizer contract of the offline dataset (milo/milo/datasets.py:6-49)."""
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
