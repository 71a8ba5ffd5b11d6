from .ism import ISM  # noqa: F401
