"""Frozen measurement constants of bench.py."""
