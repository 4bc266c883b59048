"""Action-space descriptor read by the policy / buffers (reference ``DCML_ENVs/DCML_utils/DCML_ActionSpace.py:1-9``)."""
from __future__ import annotations

import dataclasses


@dataclasses.dataclass
class Action_Space:  # noqa: N801  (reference class name: TransformerPolicy dispatches on it)
    n: int
    semi_index: int = 0
    extra: bool = False
    multi_discrete: bool = False
    high: float | None = None
    low: float | None = None
    mixed: bool = True
    continuous: bool = True

    @property
    def shape(self):
        return (self.n,)


def dcml_action_spaces(n_workers, central_execution=True, multi_agent=True, action_dim=2, extra=1):
    """``DCML_BID_FIRST_MA_ENV_SingleProcess.py:42-52``."""
    if not multi_agent:
        return [Action_Space(action_dim, semi_index=-extra, extra=True, mixed=True, low=0, high=n_workers)]
    if central_execution:
        return [Action_Space(action_dim, semi_index=-extra, extra=True)]
    return [Action_Space(action_dim, mixed=False, high=1, low=0, continuous=False)] * n_workers + \
        [Action_Space(1, mixed=False, high=1, low=0, extra=True, continuous=True)] * extra
