"""Utilities: logging, timing, profiling ranges, checkpoint/resume."""
