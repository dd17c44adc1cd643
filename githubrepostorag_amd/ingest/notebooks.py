"""Jupyter notebook de-noising (ingest/src/app/services/
jupyter_notebook_handling.py:19-193) working on the notebook JSON text (no
nbformat dependency): drop setup/dependency/filesystem/noise cells, keep
markdown, keep code as fenced python, keep outputs unless they are data dumps
(> 500 chars without table markers) or log-heavy (> 30 % log-pattern lines)."""
from __future__ import annotations

import json
import re

DEPENDENCY = [r"^!pip install", r"^!conda install", r"^!apt-get", r"^!apt install", r"^!yum install",
              r"^%pip install", r"^%conda install", r"^import sys\s*\n\s*!\{sys\.executable\}\s+-m\s+pip\s+install"]
FILESYSTEM = [r"^!mkdir", r"^!cp", r"^!mv", r"^!rm", r"^!wget", r"^!curl"]
NOISE = [r"^%matplotlib inline", r"^%config", r"^%load_ext", r"^%env", r"^!kaggle", r"^!jupyter", r"^!python -m"]
LOG_PATTERNS = [r"\d{4}-\d{2}-\d{2}\s\d{2}:\d{2}:\d{2}", r"DEBUG|INFO|WARNING|ERROR|CRITICAL", r"Downloading|Downloaded",
                r"\d+%\|[█▉▊▋▌▍▎▏ ]+\|"]
_ANSI = re.compile(r"\x1b\[[0-9;]*[A-Za-z]")


def strip_ansi(s: str) -> str:
    return _ANSI.sub("", s)


def _src(cell) -> str:
    s = cell.get("source", "")
    return "".join(s) if isinstance(s, list) else (s or "")


def _txt(v) -> str:
    return "".join(v) if isinstance(v, list) else (v or "")


def is_setup_cell(source: str) -> bool:
    pats = DEPENDENCY + FILESYSTEM + NOISE
    for line in source.split("\n"):
        line = line.strip()
        if line and any(re.match(p, line) for p in pats):
            return True
    return False


def _output_text(outputs) -> str:
    t = ""
    for o in outputs or []:
        if o.get("output_type") == "stream":
            t += _txt(o.get("text"))
        elif o.get("output_type") == "execute_result":
            t += _txt((o.get("data") or {}).get("text/plain"))
    return strip_ansi(t)


def is_output_heavy(outputs) -> bool:
    t = _output_text(outputs)
    if not t:
        return False
    if len(t) > 500:
        return not ("===" in t or "---" in t or "|" in t)
    lines = t.split("\n")
    for pat in LOG_PATTERNS:
        if re.search(pat, t):
            if sum(1 for ln in lines if re.search(pat, ln)) / max(1, len(lines)) > 0.3:
                return True
    return False


def process_notebook_text(text: str) -> str:
    nb = json.loads(text)
    cells = []
    title = (nb.get("metadata") or {}).get("title")
    if title:
        cells.append(f"# {title}\n")
    for cell in nb.get("cells", []):
        src = _src(cell)
        if not src.strip():
            continue
        if cell.get("cell_type") == "markdown":
            cells.append(src)
        elif cell.get("cell_type") == "code":
            if is_setup_cell(src):
                continue
            cells.append(f"```python\n{src}\n```")
            outs = cell.get("outputs") or []
            if outs and not is_output_heavy(outs):
                ot = _output_text(outs)
                if ot.strip():
                    cells.append(f"```\n{ot}\n```")
    return "\n\n".join(cells)
