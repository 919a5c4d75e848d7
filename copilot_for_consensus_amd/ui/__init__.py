"""Static web UI (the reference's React app, ui/src) as one dependency-free page served at /ui."""
from __future__ import annotations

from pathlib import Path

INDEX = Path(__file__).resolve().parent / "index.html"


def ui_routes(app, prefix: str = "/ui") -> None:
    from fastapi.responses import HTMLResponse, RedirectResponse

    @app.get(prefix, response_class=HTMLResponse, include_in_schema=False)
    def ui_index():
        return HTMLResponse(INDEX.read_text(encoding="utf-8"))

    @app.get("/", include_in_schema=False)
    def root():
        return RedirectResponse(prefix)
