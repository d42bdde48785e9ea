"""Reference package path ``interface`` (GTP front-end and match harness)."""
