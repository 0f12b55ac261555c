"""Column type tags accepted by ``ScalarCodec`` (stand-ins for pyspark.sql.types)."""
from __future__ import annotations

import numpy as np


class _T:
    np_dtype = np.object_
    arrow = "string"

    def __repr__(self):
        return f"{type(self).__name__}()"

    def __eq__(self, o):
        return type(self) is type(o)

    def __hash__(self):
        return hash(type(self).__name__)


class IntegerType(_T):
    np_dtype, arrow = np.int32, "int32"


class LongType(_T):
    np_dtype, arrow = np.int64, "int64"


class ShortType(_T):
    np_dtype, arrow = np.int16, "int16"


class FloatType(_T):
    np_dtype, arrow = np.float32, "float32"


class DoubleType(_T):
    np_dtype, arrow = np.float64, "float64"


class BooleanType(_T):
    np_dtype, arrow = np.bool_, "bool"


class StringType(_T):
    np_dtype, arrow = np.str_, "string"


class BinaryType(_T):
    np_dtype, arrow = np.bytes_, "binary"
