"""isaaclab_tasks import surface (registry helpers only)."""
