"""AttnLRP per-head relevance calibration."""
