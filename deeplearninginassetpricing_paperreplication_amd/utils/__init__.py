"""Auxiliary subsystems: resume checkpoints, non-finite guards, roctx tracing."""
from .checkpoint import RESUME_FILE, load_resume, save_resume
from .guards import NonFiniteError, NonFiniteMonitor
from .tracing import Timers, trace_range

__all__ = ["RESUME_FILE", "load_resume", "save_resume", "NonFiniteError", "NonFiniteMonitor",
           "Timers", "trace_range"]
