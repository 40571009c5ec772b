"""Aux subsystems: straggler/fault injection, reporting, tracing."""
from .delay import DelayModel, delay_floor
from .tracing import PhaseTimer
