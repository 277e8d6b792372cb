"""PQL: the Pilosa Query Language (grammar: reference pql/pql.peg)."""
from .ast import BETWEEN, EQ, GT, GTE, LT, LTE, NEQ, Call, Condition, Query, format_value, is_reserved_arg  # noqa: F401
from .parser import ParseError, parse_string  # noqa: F401
