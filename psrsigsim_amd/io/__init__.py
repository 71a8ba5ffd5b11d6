from .txtfile import TxtFile  # noqa: F401
