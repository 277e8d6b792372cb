"""Ported expectation of http/translator_test.go (TestTranslateStore_Reader
OK/ServerDisconnect; skipped in the reference as flaky): a client streams the
primary's key log from a byte offset and gets the reference's LogEntry
bytes.  Offset 11 skips the first entry (\\n\\x01\\x01i\\x00\\x01\\x01\\x03foo)."""
import tempfile

from pilosa_amd.server.client import InternalClient
from pilosa_amd.server.server import Server
from pilosa_amd.utils.logger import CaptureLogger


def test_translate_store_reader_from_offset():
    s = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger()).open()
    try:
        idx = s.holder.create_index_if_not_exists("i", keys=True)
        idx.create_field_if_not_exists("f")
        from pilosa_amd.server.api import QueryRequest
        s.api.query(QueryRequest("i", 'Set("foo", f=10)\nSet("bar", f=10)\nSet("baz", f=10)\n'))
        data = InternalClient().translate_data(s.uri, 11)
        assert data == b"\n\x01\x01i\x00\x01\x02\x03bar\n\x01\x01i\x00\x01\x03\x03baz"
    finally:
        s.close()
