"""Experiment surface of the reference (experiments/*), backed by the MI355X env."""
