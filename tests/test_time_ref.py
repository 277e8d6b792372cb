"""Ported expectations of the reference's time_internal_test.go (time
quantum parsing and the view-name algebra of time fields).  Each test names
the reference test it ports."""
import datetime as dt

import pytest

from pilosa_amd.models.timeq import (min_max_views, time_of_view, valid_quantum, view_by_time_unit, views_by_time,
                                     views_by_time_range)


def T(s):
    return dt.datetime.strptime(s, "%Y-%m-%d %H:%M")


def test_parse_time_quantum():  # TestParseTimeQuantum
    assert valid_quantum("YMDH")
    assert not valid_quantum("BADQUANTUM")


@pytest.mark.parametrize("unit,exp", [("Y", "F_2000"), ("M", "F_200001"), ("D", "F_20000102"), ("H", "F_2000010203")])
def test_view_by_time_unit(unit, exp):  # TestViewByTimeUnit
    assert view_by_time_unit("F", dt.datetime(2000, 1, 2, 3, 4, 5, 6), unit) == exp


def test_views_by_time():  # TestViewsByTime
    ts = dt.datetime(2000, 1, 2, 3, 4, 5, 6)
    assert views_by_time("F", ts, "YMDH") == ["F_2000", "F_200001", "F_20000102", "F_2000010203"]
    assert views_by_time("F", ts, "D") == ["F_20000102"]


def _days(prefix, y, m, d0, d1):
    return [f"{prefix}{y:04d}{m:02d}{d:02d}" for d in range(d0, d1 + 1)]


@pytest.mark.parametrize("q,start,end,exp", [
    ("Y", "2000-01-01 00:00", "2002-01-01 00:00", ["F_2000", "F_2001"]),
    ("YM", "2000-11-01 00:00", "2003-03-01 00:00", ["F_200011", "F_200012", "F_2001", "F_2002", "F_200301", "F_200302"]),
    ("YM", "2001-10-31 00:00", "2003-04-01 00:00",
     ["F_200110", "F_200111", "F_200112", "F_2002", "F_200301", "F_200302", "F_200303"]),
    ("YM", "1999-12-31 00:00", "2000-04-01 00:00", ["F_199912", "F_200001", "F_200002", "F_200003"]),
    ("YM", "2000-01-31 00:00", "2001-04-01 00:00", ["F_2000", "F_200101", "F_200102", "F_200103"]),
    ("YMD", "2000-11-28 00:00", "2003-03-02 00:00",
     ["F_20001128", "F_20001129", "F_20001130", "F_200012", "F_2001", "F_2002", "F_200301", "F_200302", "F_20030301"]),
    ("YMDH", "2000-11-28 22:00", "2002-03-01 03:00",
     ["F_2000112822", "F_2000112823", "F_20001129", "F_20001130", "F_200012", "F_2001", "F_200201", "F_200202",
      "F_2002030100", "F_2002030101", "F_2002030102"]),
    ("M", "2000-01-01 00:00", "2000-03-01 00:00", ["F_200001", "F_200002"]),
    ("MD", "2000-11-29 00:00", "2002-02-03 00:00",
     ["F_20001129", "F_20001130", "F_200012"] + [f"F_2001{m:02d}" for m in range(1, 13)] + ["F_200201", "F_20020201",
                                                                                          "F_20020202"]),
    ("MDH", "2000-11-29 22:00", "2002-03-02 03:00",
     ["F_2000112922", "F_2000112923", "F_20001130", "F_200012"] + [f"F_2001{m:02d}" for m in range(1, 13)] +
     ["F_200201", "F_200202", "F_20020301", "F_2002030200", "F_2002030201", "F_2002030202"]),
    ("D", "2000-01-01 00:00", "2000-01-04 00:00", ["F_20000101", "F_20000102", "F_20000103"]),
    ("DH", "2000-01-01 22:00", "2000-03-01 02:00",
     ["F_2000010122", "F_2000010123"] + _days("F_", 2000, 1, 2, 31) + _days("F_", 2000, 2, 1, 29) +
     ["F_2000030100", "F_2000030101"]),
    ("H", "2000-01-01 00:00", "2000-01-01 02:00", ["F_2000010100", "F_2000010101"])])
def test_views_by_time_range(q, start, end, exp):  # TestViewsByTimeRange
    assert views_by_time_range("F", T(start), T(end), q) == exp


@pytest.mark.parametrize("views,q,mn,mx", [
    ([""], "Y", "", ""), (["std_2019", "std_2020", "std_202002", "std_202002", "std_2022"], "Y", "std_2019", "std_2022"),
    (["std_201902", "std_201901"], "M", "std_201901", "std_201902"), (["std_201902", "std_201901"], "D", "", ""),
    (["std_20190201"], "D", "std_20190201", "std_20190201"), (["foo", "bar"], "D", "", "")])
def test_min_max_views(views, q, mn, mx):  # TestMinMaxViews
    assert min_max_views(views, q) == (mn, mx)


@pytest.mark.parametrize("view,exp,adj,err", [
    ("std_2019", dt.datetime(2019, 1, 1), dt.datetime(2020, 1, 1), ""),
    ("std_201902", dt.datetime(2019, 2, 1), dt.datetime(2019, 3, 1), ""),
    ("std_20190203", dt.datetime(2019, 2, 3), dt.datetime(2019, 2, 4), ""),
    ("std_2019020308", dt.datetime(2019, 2, 3, 8), dt.datetime(2019, 2, 3, 9), ""),
    ("foo", None, None, "invalid time format on view: foo"),
    ("std_201902030801", None, None, "invalid time format on view: std_201902030801")])
def test_time_of_view(view, exp, adj, err):  # TestTimeOfView
    if err:
        for a in (False, True):
            with pytest.raises(Exception, match=err):
                time_of_view(view, a)
        return
    assert time_of_view(view, False) == exp
    assert time_of_view(view, True) == adj
