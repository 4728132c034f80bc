"""Keras backend utilities: layer-name uids, clear_session, floatx."""
from __future__ import annotations

import collections
import re

_UIDS = collections.defaultdict(int)


def get_uid(prefix: str) -> int:
    _UIDS[prefix] += 1
    return _UIDS[prefix]


def unique_name(prefix: str) -> str:
    """Keras naming: first 'dense', then 'dense_1', 'dense_2', ..."""
    n = get_uid(prefix)
    return prefix if n == 1 else f"{prefix}_{n - 1}"


def clear_session() -> None:
    _UIDS.clear()


def to_snake_case(name: str) -> str:
    s = re.sub(r"(.)([A-Z][a-z]+)", r"\1_\2", name)
    s = re.sub(r"([a-z])([A-Z])", r"\1_\2", s).lower()
    return s if s[0] != "_" else "private" + s


def floatx() -> str:
    return "float32"


def image_data_format() -> str:
    return "channels_last"
