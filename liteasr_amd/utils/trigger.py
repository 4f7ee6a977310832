"""Epoch / iteration event triggers (liteasr/utils/trigger.py:6-66)."""

from functools import wraps


class Trigger(object):
    def __init__(self, interval: int, unit: str):
        assert unit in ["epoch", "iteration"]
        self.interval = interval
        self.unit = unit
        self.prev_unit = 0

    def is_triggered(self, trainer, unit: str) -> bool:
        crit = trainer.epoch if unit == "epoch" else trainer.iter
        if unit == self.unit and crit == self.prev_unit + self.interval:
            self.prev_unit += self.interval
            return True
        return False

    def __call__(self, event):
        @wraps(event)
        def wrapper(trainer, unit):
            if self.is_triggered(trainer, unit):
                event()

        return wrapper


class EventManager(object):
    def __init__(self):
        self.events = []

    def add_event(self, event):
        self.events.append(event)

    def _trigger(self, trainer, unit):
        for e in self.events:
            e(trainer, unit)

    def trigger_epoch_events(self, trainer):
        self._trigger(trainer, "epoch")

    def trigger_iteration_events(self, trainer):
        self._trigger(trainer, "iteration")
