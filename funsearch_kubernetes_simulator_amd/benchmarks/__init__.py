"""Compat namespace for the reference's `benchmarks/` package."""
