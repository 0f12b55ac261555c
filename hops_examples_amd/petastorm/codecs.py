"""Field codecs: how a Unischema field is stored in a Parquet cell.

* ``ScalarCodec(type)``            native Parquet scalar column
* ``CompressedImageCodec('png'|'jpeg', quality)``  image bytes (PIL), decoded to uint8 HxWxC
* ``NdarrayCodec()``               ``np.save`` bytes (dtype + shape preserved, any rank)
* ``CompressedNdarrayCodec()``     the same, zlib-compressed
"""
from __future__ import annotations

import io
import zlib

import numpy as np


class DataframeColumnCodec:
    def encode(self, field, value):
        raise NotImplementedError

    def decode(self, field, value):
        raise NotImplementedError

    def arrow_type(self, field) -> str:
        return "binary"


class ScalarCodec(DataframeColumnCodec):
    def __init__(self, spark_type=None):
        self.spark_type = spark_type

    def encode(self, field, value):
        return np.asarray(value, dtype=field.numpy_dtype).item() if field.numpy_dtype is not np.str_ else str(value)

    def decode(self, field, value):
        if field.numpy_dtype in (np.str_, str):
            return value
        return field.numpy_dtype(value)

    def arrow_type(self, field):
        if self.spark_type is not None and hasattr(self.spark_type, "arrow"):
            return self.spark_type.arrow
        return {np.int8: "int8", np.int16: "int16", np.int32: "int32", np.int64: "int64", np.float32: "float32",
                np.float64: "float64", np.bool_: "bool", np.uint8: "uint8"}.get(field.numpy_dtype, "string")

    def __repr__(self):
        return f"ScalarCodec({self.spark_type!r})"


class CompressedImageCodec(DataframeColumnCodec):
    def __init__(self, image_codec: str = "png", quality: int = 80):
        if image_codec not in ("png", "jpeg"):
            raise ValueError("image_codec must be 'png' or 'jpeg'")
        self.image_codec, self.quality = image_codec, quality

    def encode(self, field, value):
        from PIL import Image

        a = np.asarray(value)
        if a.dtype != np.uint8:
            raise ValueError(f"{field.name}: CompressedImageCodec needs uint8 images")
        img = Image.fromarray(a[..., 0] if a.ndim == 3 and a.shape[-1] == 1 else a)
        buf = io.BytesIO()
        if self.image_codec == "png":
            img.save(buf, format="PNG")
        else:
            img.save(buf, format="JPEG", quality=self.quality)
        return buf.getvalue()

    def decode(self, field, value):
        from PIL import Image

        a = np.asarray(Image.open(io.BytesIO(value)))
        if len(field.shape) == 3 and a.ndim == 2:
            a = a[..., None]
        return a

    def __repr__(self):
        return f"CompressedImageCodec({self.image_codec!r})"


class NdarrayCodec(DataframeColumnCodec):
    def encode(self, field, value):
        buf = io.BytesIO()
        np.save(buf, np.asarray(value, dtype=field.numpy_dtype), allow_pickle=False)
        return buf.getvalue()

    def decode(self, field, value):
        return np.load(io.BytesIO(value), allow_pickle=False)

    def __repr__(self):
        return "NdarrayCodec()"


class CompressedNdarrayCodec(NdarrayCodec):
    def encode(self, field, value):
        return zlib.compress(super().encode(field, value))

    def decode(self, field, value):
        return super().decode(field, zlib.decompress(value))

    def __repr__(self):
        return "CompressedNdarrayCodec()"
