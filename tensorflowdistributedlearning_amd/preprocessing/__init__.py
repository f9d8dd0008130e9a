"""Reference-compatible ``preprocessing`` package (see preprocessing.preprocessing)."""
