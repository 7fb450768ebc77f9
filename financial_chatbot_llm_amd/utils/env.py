"""Minimal ``.env`` loader (python-dotenv is not in the image).

Mirrors the reference's ``load_dotenv()`` call (``config.py:5``): ``KEY=VALUE`` lines, optional
``export`` prefix, quotes stripped, existing environment values win.
"""
from __future__ import annotations

import os
from typing import Optional


def load_dotenv(path: Optional[str] = None, override: bool = False) -> bool:
    path = path or os.path.join(os.getcwd(), ".env")
    if not os.path.isfile(path):
        return False
    with open(path, "r", encoding="utf-8") as fh:
        for raw in fh:
            line = raw.strip()
            if not line or line.startswith("#") or "=" not in line:
                continue
            if line.startswith("export "):
                line = line[len("export "):]
            key, val = line.split("=", 1)
            key, val = key.strip(), val.strip()
            if len(val) >= 2 and val[0] == val[-1] and val[0] in "'\"":
                val = val[1:-1]
            if override or key not in os.environ:
                os.environ[key] = val
    return True
