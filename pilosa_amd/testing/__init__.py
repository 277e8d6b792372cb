"""Test utilities shipped with the package (reference internal/test)."""
