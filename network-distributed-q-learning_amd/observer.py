"""The reference's observer plug-in point (switch_env.py:35, 48-50; observer.py:153-324), as far as a
fused device loop can honour it.

``ASyncSwitchEnv(observer=...)`` accepts the reference's only concrete observer,
``StandardObserver(delay_levels=3, delay_threshold=20)`` -- this module's stand-in, or the
reference's own ``switchfl.observer.StandardObserver`` instance (recognised by class name and
attributes) -- and hands ``delay_threshold`` to the kernels (``sfl_map_desc.delay_threshold``).
``delay_levels`` is stored but, as in the reference, unused: ``_discretize_delay`` always yields
3 levels and the observation space is built with ``n_delay_levels=3`` (observer.py:228-244, 322).
Any other observer would have to run Python inside the device loop and is refused.  The reward
function is not a plug-in in the reference (switch_env.py:48 hard-codes StandardRewardFunction).
"""
from __future__ import annotations


class StandardObserver:
    """observer.py:220-244: (switch id, semaphores, targets, discretised delays) observations."""

    def __init__(self, delay_levels: int = 3, delay_threshold: int = 20):
        self.delay_levels = delay_levels
        self.delay_threshold = delay_threshold

    def _discretize_delay(self, train, delay: int) -> int:
        available_time = train.latest_arrival - train.earliest_departure
        if delay <= 0:
            return 0
        if delay <= available_time * self.delay_threshold:
            return 1
        return 2


def delay_threshold_of(observer) -> int:
    """The kernels' delay threshold for an ``observer=`` argument (None: the reference default)."""
    if observer is None:
        return 20
    if type(observer).__name__ != "StandardObserver" or not hasattr(observer, "delay_threshold"):
        raise NotImplementedError(f"{type(observer).__name__}: only StandardObserver(delay_threshold=...) runs on "
                                  "the device path (a custom observer would run Python inside the fused loop)")
    thr = observer.delay_threshold
    if int(thr) != thr or not -65536 <= int(thr) <= 65536:
        raise ValueError(f"delay_threshold={thr!r}: the device path takes an integer in [-65536, 65536] "
                         "(observer.py:221 declares it int)")
    return int(thr)
