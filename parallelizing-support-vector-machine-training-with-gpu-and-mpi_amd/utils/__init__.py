"""Data, configuration, timing and logging utilities."""
