from .simulate import Simulation  # noqa: F401
