"""capsmi -- MI355X execution backend for CAPS relational pattern matching (host side).

Device work happens in libcapsmi.so (HIP kernels for gfx950, C ABI in include/capsmi.h); this
package mirrors CAPS's backend interface (okapi-relational .../api/table/Table.scala) over it.
"""
from . import _lib
from .expr import BOOL, F64, I64, STR
from .table import ColumnData, GpuTable, Session, StringDictionary

__all__ = ["Session", "GpuTable", "ColumnData", "StringDictionary", "I64", "BOOL", "F64", "STR", "load"]


def load():
    """Load the native library (raises ImportError if it has not been built)."""
    return _lib.load()
