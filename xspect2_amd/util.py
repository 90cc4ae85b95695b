"""Small host utilities shared by the model classes."""
from __future__ import annotations

import os
import re
import unicodedata

_QUOTES = re.compile(r"[']+")
_NUM_COMMA = re.compile(r"(?<=\d),(?=\d)")
_DISALLOWED = re.compile(r"[^-a-z0-9]+")
_DASHES = re.compile(r"-{2,}")


def slugify(text: str) -> str:
    """python-slugify's default transform for the model slugs XspecT writes
    (``probabilistic_filter_model.py:129``): NFKD -> ASCII, lower case, quotes
    dropped, digit-grouping commas dropped, other runs of non-[a-z0-9-] -> '-'."""
    text = unicodedata.normalize("NFKD", str(text)).encode("ascii", "ignore").decode("ascii")
    text = text.lower()
    text = _QUOTES.sub("", text)
    text = _NUM_COMMA.sub("", text)
    text = _DISALLOWED.sub("-", text)
    text = _DASHES.sub("-", text)
    return text.strip("-")


_DEVICE: int | None = None


def default_device() -> int:
    """GPU ordinal for banks: XSPECT2_AMD_DEVICE, else LOCAL_RANK, else 0
    (an operational setting: read at the first call, then kept)."""
    global _DEVICE
    if _DEVICE is None:
        dev = 0
        for var in ("XSPECT2_AMD_DEVICE", "LOCAL_RANK"):
            v = os.environ.get(var)
            if v is not None and v.strip():
                dev = int(v)
                break
        _DEVICE = dev
    return _DEVICE
