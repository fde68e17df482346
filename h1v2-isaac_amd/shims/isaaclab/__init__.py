"""IsaacLab import surface used by the reference scripts, backed by h12env (no Isaac Sim)."""
__version__ = "2.1.0+mi355x"
