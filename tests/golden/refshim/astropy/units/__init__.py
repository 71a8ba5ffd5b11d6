"""TEST-ONLY stand-in for the subset of ``astropy.units`` used by PsrSigSim's
filterbank synthesis path (see SURVEY.md §8(c) "Shim contract").

Used exclusively by ``tests/golden/make_golden.py`` to import the unmodified
reference from /root/reference inside the survey container and record golden
vectors.  Floating point results may differ from real astropy<4 in the last
ulp; every integer the reference derives (nsamp, Nph, nsub, ...) is therefore
recorded in the fixtures rather than re-derived.

A unit is (scale, dims) over the base dimensions (s, m, K, Jy); a Quantity is an
ndarray subclass that carries one.  Only the ufuncs/ops the path needs are
implemented.
"""
import numbers
import re

import numpy as np

_NB = 4  # s, m, K, Jy


class UnitConversionError(ValueError):
    pass


class UnitsError(UnitConversionError):
    pass


def _dims_add(a, b, sb=1.0):
    return tuple(x + sb * y for x, y in zip(a, b))


class UnitBase(object):
    __array_ufunc__ = None  # ndarray * Unit must defer to Unit.__rmul__

    def __init__(self, scale, dims, name=None):
        self.scale = float(scale)
        self.dims = tuple(float(d) for d in dims)
        self._name = name

    # ---- algebra -------------------------------------------------------
    def __mul__(self, other):
        if isinstance(other, UnitBase):
            return UnitBase(self.scale * other.scale, _dims_add(self.dims, other.dims))
        if isinstance(other, Quantity):
            return Quantity(other.view(np.ndarray), self * other.unit)
        return Quantity(other, self)

    def __rmul__(self, other):
        if isinstance(other, UnitBase):
            return other.__mul__(self)
        if isinstance(other, Quantity):
            return Quantity(other.view(np.ndarray), other.unit * self)
        return Quantity(other, self)

    def __truediv__(self, other):
        if isinstance(other, UnitBase):
            return UnitBase(self.scale / other.scale, _dims_add(self.dims, other.dims, -1.0))
        if isinstance(other, Quantity):
            return Quantity(1.0 / other.view(np.ndarray), self / other.unit)
        return Quantity(1.0 / np.asarray(other, dtype=float), self)

    def __rtruediv__(self, other):
        inv = UnitBase(1.0 / self.scale, tuple(-d for d in self.dims))
        if isinstance(other, UnitBase):
            return other * inv
        if isinstance(other, Quantity):
            return Quantity(other.view(np.ndarray), other.unit * inv)
        return Quantity(other, inv)

    def __pow__(self, p):
        p = float(p)
        return UnitBase(self.scale ** p, tuple(d * p for d in self.dims))

    def __eq__(self, other):
        try:
            other = Unit(other)
        except Exception:
            return False
        return self.dims == other.dims and np.isclose(self.scale, other.scale, rtol=1e-12, atol=0)

    def __ne__(self, other):
        return not self.__eq__(other)

    def __hash__(self):
        return hash((self.scale, self.dims))

    @property
    def physical_type(self):
        return self.dims

    def is_dimensionless(self):
        return all(d == 0 for d in self.dims)

    def to(self, other, value=1.0):
        other = Unit(other)
        if self.dims != other.dims:
            raise UnitConversionError("'{}' and '{}' are not convertible".format(self, other))
        return value * (self.scale / other.scale)

    def decompose(self):
        return UnitBase(self.scale, self.dims)

    def __repr__(self):
        return 'Unit("{}")'.format(self)

    def __str__(self):
        if self._name:
            return self._name
        names = ('s', 'm', 'K', 'Jy')
        parts = []
        for n, d in zip(names, self.dims):
            if d == 1:
                parts.append(n)
            elif d != 0:
                parts.append('{}{:g}'.format(n, d))
        s = ' '.join(parts)
        if self.scale != 1.0:
            s = '{:g} {}'.format(self.scale, s)
        return s.strip() or ''


def _base(scale, s=0, m=0, K=0, Jy=0, name=None):
    return UnitBase(scale, (s, m, K, Jy), name)


_NAMED = {
    's': _base(1.0, s=1, name='s'), 'second': _base(1.0, s=1, name='s'),
    'ms': _base(1e-3, s=1, name='ms'), 'us': _base(1e-6, s=1, name='us'),
    'microsecond': _base(1e-6, s=1, name='us'), 'ns': _base(1e-9, s=1, name='ns'),
    'min': _base(60.0, s=1, name='min'), 'h': _base(3600.0, s=1, name='h'),
    'day': _base(86400.0, s=1, name='d'), 'd': _base(86400.0, s=1, name='d'),
    'Hz': _base(1.0, s=-1, name='Hz'), 'kHz': _base(1e3, s=-1, name='kHz'),
    'MHz': _base(1e6, s=-1, name='MHz'), 'GHz': _base(1e9, s=-1, name='GHz'),
    'm': _base(1.0, m=1, name='m'), 'cm': _base(1e-2, m=1, name='cm'),
    'km': _base(1e3, m=1, name='km'),
    'pc': _base(3.0856775814913673e16, m=1, name='pc'),
    'K': _base(1.0, K=1, name='K'), 'Jy': _base(1.0, Jy=1, name='Jy'),
    'mJy': _base(1e-3, Jy=1, name='mJy'),
    '': _base(1.0, name=''), 'dimensionless': _base(1.0, name=''),
}

_TOKEN = re.compile(r'\s*([A-Za-z]+)\s*(?:(?:\^|\*\*)\s*(-?[0-9.]+))?\s*')


def _parse(s):
    s = s.strip()
    if s in _NAMED:
        return _NAMED[s]
    unit = _NAMED['']
    op = '*'
    pos = 0
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise ValueError("cannot parse unit {!r}".format(s))
        name, exp = m.group(1), m.group(2)
        if name not in _NAMED:
            raise ValueError("unknown unit {!r}".format(name))
        u = _NAMED[name] ** (float(exp) if exp else 1.0)
        unit = unit * u if op == '*' else unit / u
        pos = m.end()
        if pos < len(s):
            op = s[pos]
            if op not in '*/':
                raise ValueError("cannot parse unit {!r}".format(s))
            pos += 1
    return unit


def Unit(x):
    if isinstance(x, UnitBase):
        return x
    if isinstance(x, str):
        return _parse(x)
    if isinstance(x, Quantity) and x.shape == ():
        return UnitBase(float(x.view(np.ndarray)) * x.unit.scale, x.unit.dims)
    if isinstance(x, numbers.Number):
        return UnitBase(float(x), (0,) * _NB)
    raise TypeError("cannot make a unit from {!r}".format(x))


class _Core(object):
    Unit = staticmethod(Unit)
    UnitBase = UnitBase
    UnitConversionError = UnitConversionError


core = _Core()
dimensionless_unscaled = _NAMED['']
for _k, _v in _NAMED.items():
    if _k:
        globals()[_k] = _v


def _as_unit(x):
    return x.unit if isinstance(x, Quantity) else dimensionless_unscaled


def _raw(x):
    return x.view(np.ndarray) if isinstance(x, Quantity) else x


class Quantity(np.ndarray):
    def __new__(cls, value, unit=None, dtype=None, copy=True):
        unit = dimensionless_unscaled if unit is None else Unit(unit)
        if isinstance(value, Quantity):
            if unit is not dimensionless_unscaled:
                value = value.to(unit)
                return value
            return value.copy() if copy else value
        if dtype is None:
            arr = np.array(value, dtype=float, copy=True)
        else:
            arr = np.array(value, dtype=dtype, copy=True)
        obj = arr.view(cls)
        obj._unit = unit
        return obj

    def __array_finalize__(self, obj):
        self._unit = getattr(obj, '_unit', dimensionless_unscaled)

    # ---- basic properties ---------------------------------------------
    @property
    def unit(self):
        return self._unit

    @property
    def value(self):
        v = self.view(np.ndarray)
        return v if v.shape else v[()]

    def to(self, unit):
        unit = Unit(unit)
        fac = self._unit.to(unit)
        return Quantity(self.view(np.ndarray) * fac, unit)

    def to_value(self, unit=None):
        if unit is None:
            return self.value
        return self.to(unit).value

    def decompose(self):
        return Quantity(self.view(np.ndarray) * self._unit.scale,
                        UnitBase(1.0, self._unit.dims))

    def _dimless_value(self):
        if not self._unit.is_dimensionless():
            raise TypeError("only dimensionless scalar quantities can be converted to Python scalars")
        return self.view(np.ndarray) * self._unit.scale

    def __float__(self):
        return float(self._dimless_value())

    def __int__(self):
        return int(self._dimless_value())

    def __index__(self):
        return int(self._dimless_value())

    def __bool__(self):
        return bool(self.view(np.ndarray).all() if self.shape else self.view(np.ndarray))

    def __getitem__(self, key):
        out = super().__getitem__(key)
        if not isinstance(out, Quantity):
            out = Quantity(out, self._unit)
        return out

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]

    def __eq__(self, other):
        if other is None:
            return False
        return np.equal(self, other)

    def __ne__(self, other):
        if other is None:
            return True
        return np.not_equal(self, other)

    __hash__ = None

    def __repr__(self):
        return '<Quantity {} {}>'.format(self.view(np.ndarray), self._unit)

    def __str__(self):
        return '{} {}'.format(self.view(np.ndarray), self._unit)

    def __format__(self, spec):
        v = self.view(np.ndarray)
        if v.shape == ():
            return format(float(v), spec) + ' ' + str(self._unit)
        return str(self)

    def __reduce__(self):
        raise TypeError("shim Quantity is not picklable")

    # ---- numpy protocol ------------------------------------------------
    def __array_ufunc__(self, ufunc, method, *inputs, **kwargs):
        out = kwargs.pop('out', None)
        name = ufunc.__name__
        raw_in = [_raw(x) for x in inputs]
        units = [_as_unit(x) for x in inputs]
        is_q = [isinstance(x, Quantity) for x in inputs]

        if method == 'reduce':
            res = getattr(ufunc, method)(raw_in[0], **kwargs)
            ru = units[0] if name in ('add', 'maximum', 'minimum') else dimensionless_unscaled
            return self._wrap(res, ru, out)
        if method != '__call__':
            return NotImplemented

        def convert_to(x, u_from, u_to, q):
            if not q:
                # bare numbers: allowed against dimensionless, or when all zero
                if u_to.is_dimensionless():
                    return np.asarray(x, dtype=float) / u_to.scale
                if np.all(np.asarray(x) == 0):
                    return x
                raise UnitConversionError("cannot combine bare number with {}".format(u_to))
            return x * u_from.to(u_to)

        if name in ('multiply',):
            return self._wrap(raw_in[0] * raw_in[1], units[0] * units[1], out)
        if name in ('true_divide', 'divide'):
            return self._wrap(raw_in[0] / raw_in[1], units[0] / units[1], out)
        if name == 'reciprocal':
            return self._wrap(1.0 / raw_in[0], dimensionless_unscaled / units[0], out)
        if name == 'power':
            p = inputs[1]
            if isinstance(p, Quantity):
                p = float(p)
            return self._wrap(raw_in[0] ** p, units[0] ** float(np.asarray(p)), out)
        if name == '_ones_like':
            return self._wrap(np.ones_like(raw_in[0]), dimensionless_unscaled, out)
        if name == 'sqrt':
            return self._wrap(np.sqrt(raw_in[0]), units[0] ** 0.5, out)
        if name == 'square':
            return self._wrap(raw_in[0] ** 2, units[0] ** 2, out)
        if name in ('negative', 'absolute', 'positive', 'fabs', 'rint', 'floor', 'ceil'):
            return self._wrap(ufunc(raw_in[0]), units[0], out)
        if name in ('add', 'subtract', 'remainder', 'fmod', 'maximum', 'minimum',
                    'equal', 'not_equal', 'less', 'less_equal', 'greater',
                    'greater_equal', 'floor_divide'):
            # convert everything to the unit of the first Quantity operand
            ref = units[0] if is_q[0] else units[1]
            a = convert_to(raw_in[0], units[0], ref, is_q[0])
            b = convert_to(raw_in[1], units[1], ref, is_q[1])
            res = ufunc(a, b)
            if name in ('equal', 'not_equal', 'less', 'less_equal', 'greater', 'greater_equal'):
                return res
            if name == 'floor_divide':
                return self._wrap(res, dimensionless_unscaled, out)
            return self._wrap(res, ref, out)
        if name in ('exp', 'log', 'log10', 'log2', 'sin', 'cos', 'tan', 'expm1', 'log1p'):
            x = raw_in[0] * units[0].scale if is_q[0] else raw_in[0]
            if is_q[0] and not units[0].is_dimensionless():
                raise UnitsError("{} requires a dimensionless argument".format(name))
            return self._wrap(ufunc(x), dimensionless_unscaled, out)
        if name in ('isfinite', 'isnan', 'isinf', 'signbit'):
            return ufunc(raw_in[0])
        raise NotImplementedError("shim Quantity does not support ufunc {}".format(name))

    def _wrap(self, res, unit, out):
        if out is not None:
            tgt = out[0] if isinstance(out, tuple) else out
            if isinstance(tgt, Quantity):
                tgt.view(np.ndarray)[...] = res * unit.to(tgt.unit) if unit.dims == tgt.unit.dims else res
                return tgt
            # a plain ndarray ``out`` also arrives through numpy's temporary
            # elision (numpy>=2 elides ``q * big_temporary`` in place); keep
            # the unit by returning a Quantity view of the buffer.
            tgt[...] = res
            q = tgt.view(Quantity)
            q._unit = unit
            return q
        q = np.asarray(res).view(Quantity)
        q._unit = unit
        return q

    def __array_function__(self, func, types, args, kwargs):
        name = func.__name__
        if name in ('sum', 'amax', 'amin', 'max', 'min', 'mean', 'round', 'around',
                    'copy', 'reshape', 'append', 'concatenate', 'squeeze', 'ravel',
                    'linspace', 'where', 'shape', 'ndim', 'size', 'atleast_1d',
                    'broadcast_to', 'diff', 'cumsum', 'argmax', 'argmin', 'tile',
                    'array_equal', 'isclose', 'allclose', 'zeros_like', 'ones_like',
                    'empty_like', 'full_like', 'result_type', 'can_cast', 'trapz',
                    'trapezoid'):
            return super().__array_function__(func, types, args, kwargs)
        return super().__array_function__(func, types, args, kwargs)

    def round(self, decimals=0, out=None):
        return self._wrap(np.round(self.view(np.ndarray), decimals), self._unit, out)


def quantity_input(*a, **k):  # pragma: no cover - decorator stub
    def deco(f):
        return f
    return deco
