"""JSON bodies byte-compatible with Go's encoding/json (what the reference's
HTTP handlers write, http/handler.go json.NewEncoder(w).Encode): compact
separators, UTF-8 text left unescaped, and the HTML-safe escapes Go applies
to '<', '>', '&', U+2028 and U+2029.  ``encode_line`` adds the trailing
newline json.Encoder writes."""
from __future__ import annotations

import json

_ESC = (("<", "\\u003c"), (">", "\\u003e"), ("&", "\\u0026"), ("\u2028", "\\u2028"), ("\u2029", "\\u2029"))


def dumps(obj) -> str:
    s = json.dumps(obj, separators=(",", ":"), ensure_ascii=False)
    for a, b in _ESC:
        if a in s:   # only string contents can hold these: structural JSON never does
            s = s.replace(a, b)
    return s


def encode_line(obj) -> str:
    return dumps(obj) + "\n"
