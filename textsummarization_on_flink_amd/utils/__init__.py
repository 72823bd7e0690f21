"""Utilities: logging setup (``logs``), ``--debug`` non-finite tensor watch (``debug``)."""
from .debug import NonFiniteWatch, nonfinite_report
from .logs import project_root, setup_logging

__all__ = ["NonFiniteWatch", "nonfinite_report", "project_root", "setup_logging"]
