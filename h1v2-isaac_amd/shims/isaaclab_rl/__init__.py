"""isaaclab_rl import surface (rsl_rl integration only)."""
