"""rsl_rl import surface backed by h12env.ppo (rsl-rl-lib 2.3 semantics)."""
__version__ = "2.3.3+mi355x"
