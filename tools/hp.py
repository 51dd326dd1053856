"""High-precision (Decimal, ~60 digits) scalar math used by the table generators.

Only the generators under tools/ use this; nothing on the product or test path imports it.
"""
from decimal import Decimal, getcontext

getcontext().prec = 70
D = Decimal

_PI = None


def pi():
    """pi by the Machin formula."""
    global _PI
    if _PI is None:
        getcontext().prec += 10
        _PI = 4 * (4 * _atan_small(D(1) / 5) - _atan_small(D(1) / 239))
        getcontext().prec -= 10
        _PI = +_PI
    return _PI


def _atan_small(x):
    # Taylor series, |x| small
    x = D(x)
    x2 = x * x
    term = x
    s = x
    n = 1
    eps = D(10) ** (-(getcontext().prec + 5))
    while True:
        term *= -x2
        n += 2
        t = term / n
        if abs(t) < eps:
            break
        s += t
    return s


def sin(x):
    x = D(x)
    p2 = 2 * pi()
    x = x - p2 * (x / p2).to_integral_value()
    getcontext().prec += 10
    x2 = x * x
    term = x
    s = x
    n = 1
    eps = D(10) ** (-(getcontext().prec + 5))
    while abs(term) > eps:
        term *= -x2 / ((n + 1) * (n + 2))
        n += 2
        s += term
    getcontext().prec -= 10
    return +s


def cos(x):
    x = D(x)
    p2 = 2 * pi()
    x = x - p2 * (x / p2).to_integral_value()
    getcontext().prec += 10
    x2 = x * x
    term = D(1)
    s = D(1)
    n = 0
    eps = D(10) ** (-(getcontext().prec + 5))
    while abs(term) > eps:
        term *= -x2 / ((n + 1) * (n + 2))
        n += 2
        s += term
    getcontext().prec -= 10
    return +s


def sqrt(x):
    return D(x).sqrt()


def atan(x):
    x = D(x)
    if x < 0:
        return -atan(-x)
    if x > 1:
        return pi() / 2 - atan(1 / x)
    # argument halving: atan(x) = 2 atan(x / (1 + sqrt(1 + x^2)))
    k = 0
    while x > D("0.1"):
        x = x / (1 + (1 + x * x).sqrt())
        k += 1
    return _atan_small(x) * (2 ** k)


def atan2(y, x):
    y = D(y)
    x = D(x)
    if x > 0:
        return atan(y / x)
    if x < 0:
        return atan(y / x) + (pi() if y >= 0 else -pi())
    if y > 0:
        return pi() / 2
    if y < 0:
        return -pi() / 2
    return D(0)


def asin(x):
    x = D(x)
    return atan2(x, (1 - x * x).sqrt())


def acos(x):
    x = D(x)
    return atan2((1 - x * x).sqrt(), x)


def tan(x):
    return sin(x) / cos(x)


def to_double(x):
    """Correctly rounded conversion to an IEEE double."""
    return float(D(x))
