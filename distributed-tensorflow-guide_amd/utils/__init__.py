"""Utilities: timing, profiling markers, metrics."""
