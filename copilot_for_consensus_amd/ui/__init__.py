"""Static web UI (the reference's React app, ui/src) as one dependency-free page served at /ui."""
from __future__ import annotations

import json
from pathlib import Path

INDEX = Path(__file__).resolve().parent / "index.html"


def render_index(bases: dict | None = None) -> str:
    """The page, told where the reporting / ingestion / auth APIs live (default: the gateway layout)."""
    html = INDEX.read_text(encoding="utf-8")
    if bases:
        inject = f"<script>window.CFC_BASES = {json.dumps(bases)};</script>\n<script>"
        html = html.replace("<script>", inject, 1)
    return html


def ui_routes(app, prefix: str = "/ui", bases: dict | None = None) -> None:
    from fastapi.responses import HTMLResponse, RedirectResponse
    page = render_index(bases)

    @app.get(prefix, response_class=HTMLResponse, include_in_schema=False)
    def ui_index():
        return HTMLResponse(page)

    @app.get("/", include_in_schema=False)
    def root():
        return RedirectResponse(prefix)
