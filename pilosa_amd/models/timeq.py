"""Time quantums and time views (reference: time.go).

A time field with quantum e.g. ``YMDH`` writes every timestamped bit into one
view per unit (``standard_2019``, ``standard_201901``, ``standard_20190102``,
``standard_2019010215``).  A range query ``[from, to)`` is answered from the
minimal covering set of views (:func:`views_by_time_range`, time.go:104-181),
which the GPU path turns into one N-way OR program over those views.
"""
from __future__ import annotations

import datetime as dt
from typing import List, Tuple

TIME_FORMAT = "%Y-%m-%dT%H:%M"
VALID_QUANTUMS = ("Y", "YM", "YMD", "YMDH", "M", "MD", "MDH", "D", "DH", "H", "")


class InvalidTimeQuantum(ValueError):
    pass


def valid_quantum(q: str) -> bool:
    return q in VALID_QUANTUMS


def _go_add_date(t: dt.datetime, years=0, months=0, days=0) -> dt.datetime:
    """Go time.AddDate semantics (normalises overflowing days)."""
    total = t.year * 12 + (t.month - 1) + months + 12 * years
    y, m = divmod(total, 12)
    base = dt.datetime(y, m + 1, 1, t.hour, t.minute, t.second, t.microsecond)
    return base + dt.timedelta(days=t.day - 1 + days)


def _add_month(t: dt.datetime) -> dt.datetime:
    if t.day > 28:
        t = dt.datetime(t.year, t.month, 1, t.hour)
    return _go_add_date(t, months=1)


def view_by_time_unit(name: str, t: dt.datetime, unit: str) -> str:
    if unit == "Y":
        return f"{name}_{t.year:04d}"
    if unit == "M":
        return f"{name}_{t.year:04d}{t.month:02d}"
    if unit == "D":
        return f"{name}_{t.year:04d}{t.month:02d}{t.day:02d}"
    if unit == "H":
        return f"{name}_{t.year:04d}{t.month:02d}{t.day:02d}{t.hour:02d}"
    return ""


def views_by_time(name: str, t: dt.datetime, q: str) -> List[str]:
    return [v for v in (view_by_time_unit(name, t, u) for u in q) if v]


def _next_year_gte(t, end):
    nxt = _go_add_date(t, years=1)
    if nxt.year == end.year:
        return True
    return end > nxt


def _next_month_gte(t, end):
    nxt = _go_add_date(t, months=1)
    if nxt.year == end.year and nxt.month == end.month:
        return True
    return end > nxt


def _next_day_gte(t, end):
    nxt = _go_add_date(t, days=1)
    if (nxt.year, nxt.month, nxt.day) == (end.year, end.month, end.day):
        return True
    return end > nxt


def views_by_time_range(name: str, start: dt.datetime, end: dt.datetime, q: str) -> List[str]:
    t = start
    has_y, has_m, has_d, has_h = "Y" in q, "M" in q, "D" in q, "H" in q
    out: List[str] = []
    if has_h or has_d or has_m:
        while t < end:
            if has_h:
                if not _next_day_gte(t, end):
                    break
                if t.hour != 0:
                    out.append(view_by_time_unit(name, t, "H"))
                    t = t + dt.timedelta(hours=1)
                    continue
            if has_d:
                if not _next_month_gte(t, end):
                    break
                if t.day != 1:
                    out.append(view_by_time_unit(name, t, "D"))
                    t = _go_add_date(t, days=1)
                    continue
            if has_m:
                if not _next_year_gte(t, end):
                    break
                if t.month != 1:
                    out.append(view_by_time_unit(name, t, "M"))
                    t = _add_month(t)
                    continue
            break
    while t < end:
        if has_y and _next_year_gte(t, end):
            out.append(view_by_time_unit(name, t, "Y"))
            t = _go_add_date(t, years=1)
        elif has_m and _next_month_gte(t, end):
            out.append(view_by_time_unit(name, t, "M"))
            t = _add_month(t)
        elif has_d and _next_day_gte(t, end):
            out.append(view_by_time_unit(name, t, "D"))
            t = _go_add_date(t, days=1)
        elif has_h:
            out.append(view_by_time_unit(name, t, "H"))
            t = t + dt.timedelta(hours=1)
        else:
            break
    return out


def parse_time(v) -> dt.datetime:
    """time.go:220 parseTime: 'YYYY-MM-DDTHH:MM' string or unix seconds."""
    if isinstance(v, str):
        try:
            return dt.datetime.strptime(v, TIME_FORMAT)
        except ValueError:
            raise ValueError("cannot parse string time")
    if isinstance(v, int) and not isinstance(v, bool):
        return dt.datetime.utcfromtimestamp(v)
    raise ValueError("arg must be a timestamp")


def view_time_part(v: str) -> str:
    return v.split("_")[-1]


def min_max_views(views: List[str], q: str) -> Tuple[str, str]:
    views = sorted(views)
    chars = 4 if "Y" in q else 6 if "M" in q else 8 if "D" in q else 10 if "H" in q else 0
    mn = next((v for v in views if len(view_time_part(v)) == chars), "")
    mx = next((v for v in reversed(views) if len(view_time_part(v)) == chars), "")
    return mn, mx


def time_of_view(v: str, adj: bool) -> dt.datetime:
    if not v:
        return dt.datetime(1, 1, 1)
    tp = view_time_part(v)
    if len(tp) == 4:
        t = dt.datetime(int(tp), 1, 1)
        return _go_add_date(t, years=1) if adj else t
    if len(tp) == 6:
        t = dt.datetime(int(tp[:4]), int(tp[4:6]), 1)
        return _add_month(t) if adj else t
    if len(tp) == 8:
        t = dt.datetime(int(tp[:4]), int(tp[4:6]), int(tp[6:8]))
        return _go_add_date(t, days=1) if adj else t
    if len(tp) == 10:
        t = dt.datetime(int(tp[:4]), int(tp[4:6]), int(tp[6:8]), int(tp[8:10]))
        return t + dt.timedelta(hours=1) if adj else t
    raise ValueError(f"invalid time format on view: {v}")
