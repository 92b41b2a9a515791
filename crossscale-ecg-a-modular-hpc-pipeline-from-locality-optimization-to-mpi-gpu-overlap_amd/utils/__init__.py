"""Utilities: CSV schemas, timing (hipEvent), logging, profiling ranges, checkpointing, config."""
