"""Evaluation: token streams, sliding-window PPL, sweeps."""
