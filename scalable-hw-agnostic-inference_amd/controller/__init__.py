"""Control loops."""
