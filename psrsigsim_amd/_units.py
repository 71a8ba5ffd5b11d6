"""Minimal physical-units layer for the API surface.

The reference threads astropy Quantities through every call
(``utils/utils.py:310-340`` make_quant).  This engine computes in plain float64
in fixed working units (MHz, s, ms for delays, Jy, K, m) and only exposes
Quantities at the API boundary so that user code written against the
reference (``sig.tobs.value``, ``make_quant(5, 'ms')``, ``psr.period.to('ms')``)
keeps working.  A unit is a scale (to SI-like base units) and a dimension
vector over (s, m, K, Jy).
"""
import numbers
import re

import numpy as np

__all__ = ["Unit", "Quantity", "make_quant", "UnitConversionError", "to_value"]


class UnitConversionError(ValueError):
    pass


class Unit(object):
    __array_ufunc__ = None  # ndarray * Unit -> Unit.__rmul__

    def __init__(self, scale=1.0, dims=(0, 0, 0, 0), name=None):
        self.scale = float(scale)
        self.dims = tuple(float(d) for d in dims)
        self.name = name

    def __mul__(self, o):
        if isinstance(o, Unit):
            return Unit(self.scale * o.scale, [a + b for a, b in zip(self.dims, o.dims)])
        return Quantity(o, self)

    def __rmul__(self, o):
        return Quantity(o, self)

    def __truediv__(self, o):
        if isinstance(o, Unit):
            return Unit(self.scale / o.scale, [a - b for a, b in zip(self.dims, o.dims)])
        return Quantity(1.0 / np.asarray(o, dtype=float), self)

    def __rtruediv__(self, o):
        return Quantity(o, self ** -1)

    def __pow__(self, p):
        return Unit(self.scale ** p, [d * p for d in self.dims])

    def __eq__(self, o):
        try:
            o = as_unit(o)
        except (TypeError, ValueError):
            return False
        return self.dims == o.dims and abs(self.scale - o.scale) <= 1e-12 * abs(o.scale)

    def __hash__(self):
        return hash(self.dims)

    def factor_to(self, o):
        o = as_unit(o)
        if self.dims != o.dims:
            raise UnitConversionError("'%s' and '%s' are not convertible" % (self, o))
        return self.scale / o.scale

    def is_dimensionless(self):
        return not any(self.dims)

    def __str__(self):
        if self.name is not None:
            return self.name
        parts = []
        for n, d in zip(("s", "m", "K", "Jy"), self.dims):
            if d:
                parts.append(n if d == 1 else "%s%g" % (n, d))
        s = " ".join(parts)
        return ("%g %s" % (self.scale, s)).strip() if self.scale != 1.0 else s

    __repr__ = __str__


def _u(scale, s=0, m=0, K=0, Jy=0, name=None):
    return Unit(scale, (s, m, K, Jy), name)


UNITS = {
    "": _u(1.0, name=""), "s": _u(1.0, s=1, name="s"), "second": _u(1.0, s=1, name="s"),
    "ms": _u(1e-3, s=1, name="ms"), "us": _u(1e-6, s=1, name="us"),
    "microsecond": _u(1e-6, s=1, name="us"), "ns": _u(1e-9, s=1, name="ns"),
    "min": _u(60.0, s=1, name="min"), "h": _u(3600.0, s=1, name="h"),
    "day": _u(86400.0, s=1, name="d"), "d": _u(86400.0, s=1, name="d"),
    "Hz": _u(1.0, s=-1, name="Hz"), "kHz": _u(1e3, s=-1, name="kHz"),
    "MHz": _u(1e6, s=-1, name="MHz"), "GHz": _u(1e9, s=-1, name="GHz"),
    "m": _u(1.0, m=1, name="m"), "cm": _u(1e-2, m=1, name="cm"), "km": _u(1e3, m=1, name="km"),
    "pc": _u(3.0856775814913673e16, m=1, name="pc"),
    "K": _u(1.0, K=1, name="K"), "Jy": _u(1.0, Jy=1, name="Jy"), "mJy": _u(1e-3, Jy=1, name="mJy"),
}
_TOK = re.compile(r"\s*([A-Za-z]+)\s*(?:(?:\^|\*\*)\s*(-?[0-9.]+))?\s*")


_PARSED = {}


def as_unit(x):
    if isinstance(x, Unit):
        return x
    if isinstance(x, str):
        u = UNITS.get(x)
        if u is None:
            u = _PARSED.get(x)
        if u is None:
            u = _PARSED[x] = _parse_unit(x)      # compound strings parsed once per process
        return u
    raise TypeError("not a unit: %r" % (x,))


def _parse_unit(x):
    s = x.strip()
    if s in UNITS:
        return UNITS[s]
    out, op, pos = UNITS[""], "*", 0
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.group(1) not in UNITS:
            raise ValueError("cannot parse unit %r" % x)
        u = UNITS[m.group(1)] ** (float(m.group(2)) if m.group(2) else 1.0)
        out = out * u if op == "*" else out / u
        pos = m.end()
        if pos < len(s):
            op = s[pos]
            if op not in "*/":
                raise ValueError("cannot parse unit %r" % x)
            pos += 1
    out.name = s
    return out


class Quantity(object):
    """value (float or ndarray) in ``unit``."""
    __array_priority__ = 1000

    def __init__(self, value, unit=""):
        t = type(value)
        if t is float or t is int:
            self._value = float(value)        # (the common scalar case, without numpy)
        else:
            if isinstance(value, Quantity):
                value = value.to(unit).value if unit != "" else value.value
            self._value = np.asarray(value, dtype=float) if np.ndim(value) else float(value)
        self.unit = as_unit(unit)

    # -- access --------------------------------------------------------
    @property
    def value(self):
        return self._value

    def to(self, unit):
        unit = as_unit(unit)
        return Quantity(self._value * self.unit.factor_to(unit), unit)

    def to_value(self, unit=None):
        return self._value if unit is None else self.to(unit).value

    def decompose(self):
        return Quantity(self._value * self.unit.scale, Unit(1.0, self.unit.dims))

    def __array__(self, dtype=None, copy=None):
        return np.asarray(self._value, dtype=dtype)

    def __len__(self):
        return len(self._value)

    def __getitem__(self, i):
        return Quantity(np.asarray(self._value)[i], self.unit)

    def __iter__(self):
        for v in np.asarray(self._value):
            yield Quantity(v, self.unit)

    @property
    def shape(self):
        return np.shape(self._value)

    def _dimless(self):
        if not self.unit.is_dimensionless():
            raise TypeError("only dimensionless quantities convert to Python scalars")
        return self._value * self.unit.scale

    def __float__(self):
        return float(self._dimless())

    def __int__(self):
        return int(self._dimless())

    # -- arithmetic ----------------------------------------------------
    def _other(self, o):
        """o expressed in self's unit (for +, -, comparisons)."""
        if isinstance(o, Quantity):
            return o._value * o.unit.factor_to(self.unit)
        if self.unit.is_dimensionless():
            return np.asarray(o, dtype=float) / self.unit.scale
        if np.all(np.asarray(o) == 0):
            return o
        raise UnitConversionError("cannot combine a bare number with %s" % self.unit)

    def __add__(self, o):
        return Quantity(self._value + self._other(o), self.unit)

    __radd__ = __add__

    def __sub__(self, o):
        return Quantity(self._value - self._other(o), self.unit)

    def __rsub__(self, o):
        return Quantity(self._other(o) - self._value, self.unit)

    def __neg__(self):
        return Quantity(-self._value, self.unit)

    def __mul__(self, o):
        if isinstance(o, Quantity):
            return Quantity(self._value * o._value, self.unit * o.unit)
        if isinstance(o, Unit):
            return Quantity(self._value, self.unit * o)
        return Quantity(self._value * np.asarray(o, dtype=float), self.unit)

    __rmul__ = __mul__

    def __truediv__(self, o):
        if isinstance(o, Quantity):
            return Quantity(self._value / o._value, self.unit / o.unit)
        if isinstance(o, Unit):
            return Quantity(self._value, self.unit / o)
        return Quantity(self._value / np.asarray(o, dtype=float), self.unit)

    def __rtruediv__(self, o):
        return Quantity(np.asarray(o, dtype=float) / self._value, self.unit ** -1)

    def __pow__(self, p):
        return Quantity(self._value ** float(p), self.unit ** float(p))

    def __mod__(self, o):
        return Quantity(np.remainder(self._value, self._other(o)), self.unit)

    def __floordiv__(self, o):
        return Quantity(np.floor_divide(self._value, self._other(o)), "")

    def _cmp(self, o, op):
        if o is None:
            return op is np.not_equal
        return op(self._value, self._other(o))

    def __eq__(self, o):
        return self._cmp(o, np.equal)

    def __ne__(self, o):
        return self._cmp(o, np.not_equal)

    def __lt__(self, o):
        return self._cmp(o, np.less)

    def __le__(self, o):
        return self._cmp(o, np.less_equal)

    def __gt__(self, o):
        return self._cmp(o, np.greater)

    def __ge__(self, o):
        return self._cmp(o, np.greater_equal)

    __hash__ = None

    def __repr__(self):
        return "<Quantity %s %s>" % (self._value, self.unit)

    def __str__(self):
        return "%s %s" % (self._value, self.unit)

    def __format__(self, spec):
        if np.ndim(self._value) == 0:
            return format(float(self._value), spec) + " " + str(self.unit)
        return str(self)


def make_quant(param, default_unit):
    """utils/utils.py:310-340: attach ``default_unit`` to a bare number; a
    Quantity is checked for convertibility (ValueError otherwise) and returned
    unchanged."""
    unit = as_unit(default_unit)
    if isinstance(param, Quantity):
        try:
            param.to(unit)
        except UnitConversionError:
            raise ValueError("Quantity {0} with incompatible unit {1}".format(param, default_unit))
        return param
    return Quantity(param, unit)


def to_value(x, unit):
    """Float(s) of ``x`` in ``unit`` (bare numbers are taken to be in it)."""
    if isinstance(x, Quantity):
        return x.to(unit).value
    return x
