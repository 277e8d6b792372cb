"""Ported expectations of inmem/translator_test.go (an in-memory translate
store: per-index column ids and per-(index, field) row ids, each starting at
1) and gopsutil/systeminfo_test.go (host facts for diagnostics)."""
from pilosa_amd.models.translate import TranslateFile
from pilosa_amd.utils.sysinfo import SystemInfo


def _mem_store():
    return TranslateFile().open()    # no path: the in-memory store


def test_translate_column():  # TestTranslateStore_TranslateColumn
    s = _mem_store()
    try:
        assert s.translate_columns_to_uint64("IDX0", ["foo"]) == [1]
        assert s.translate_columns_to_uint64("IDX0", ["bar"]) == [2]
        assert s.translate_columns_to_uint64("IDX1", ["bar"]) == [1]
        assert s.translate_column_to_string("IDX0", 2) == "bar"
    finally:
        s.close()


def test_translate_row():  # TestTranslateStore_TranslateRow
    s = _mem_store()
    try:
        assert s.translate_rows_to_uint64("IDX0", "FRAME0", ["foo"]) == [1]
        assert s.translate_rows_to_uint64("IDX0", "FRAME0", ["bar"]) == [2]
        assert s.translate_rows_to_uint64("IDX1", "FRAME0", ["bar"]) == [1]
        assert s.translate_rows_to_uint64("IDX0", "FRAME1", ["bar"]) == [1]
        assert s.translate_row_to_string("IDX0", "FRAME0", 2) == "bar"
    finally:
        s.close()


def test_system_info():  # TestSystemInfo
    si = SystemInfo()
    assert si.uptime() > 0
    assert isinstance(si.platform(), str) and isinstance(si.family(), str)
    assert isinstance(si.os_version(), str) and isinstance(si.kernel_version(), str)
    assert si.mem_free() >= 0 and si.mem_used() >= 0 and si.mem_total() > 0
    assert si.cpu_arch() != ""
    d = si.to_dict()
    assert d["cpuArch"] and d["memoryFree"] >= 0
