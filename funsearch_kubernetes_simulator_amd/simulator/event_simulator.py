"""Compat path for `simulator/event_simulator.py` (reference); see .events."""
from .events import DiscreteEventSimulator, Event, EventType  # noqa: F401

__all__ = ["DiscreteEventSimulator", "Event", "EventType"]
