"""Periodic training events (behaviour of liteasr/utils/trigger.py:6-66).

``Trigger(interval, unit)`` wraps a zero-argument callable (e.g. ``trainer.valid``) into
an event ``event(trainer, unit)`` that fires when the trainer's counter for ``unit``
(``trainer.epoch`` or ``trainer.iter``) reaches the next multiple of ``interval``;
``EventManager`` holds the events and the Trainer pokes it once per epoch boundary and
once per optimizer step.
"""

from functools import update_wrapper

_COUNTERS = {"epoch": "epoch", "iteration": "iter"}


class Trigger(object):
    def __init__(self, interval: int, unit: str):
        assert unit in _COUNTERS, f"unit must be one of {sorted(_COUNTERS)}"
        self.interval = interval
        self.unit = unit
        self.prev_unit = 0  # counter value at the last firing

    def is_triggered(self, trainer, unit: str) -> bool:
        if unit != self.unit:
            return False
        due = self.prev_unit + self.interval
        if getattr(trainer, _COUNTERS[unit]) != due:
            return False
        self.prev_unit = due
        return True

    def __call__(self, action):
        trigger = self

        def event(trainer, unit):
            if trigger.is_triggered(trainer, unit):
                action()

        return update_wrapper(event, action)


class EventManager(object):
    def __init__(self):
        self.events = []

    def add_event(self, event):
        self.events.append(event)

    def _fire(self, trainer, unit):
        for event in list(self.events):
            event(trainer, unit)

    def trigger_epoch_events(self, trainer):
        self._fire(trainer, "epoch")

    def trigger_iteration_events(self, trainer):
        self._fire(trainer, "iteration")
