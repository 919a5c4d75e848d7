"""Diffs between two revisions of an Internet-Draft.

Parity target: adapters/copilot_draft_diff (DraftDiff models.py, DraftDiffProvider.getdiff
provider.py:19, DatatrackerDiffProvider datatracker_provider.py:10, MockDiffProvider
mock_provider.py:10 with predefined diffs and text/markdown/html mock content, factory.py:28).

The reference's Datatracker provider is a stub that raises NotImplementedError; here it works:
both revisions' plain text are fetched from the IETF archive (``{base_url}/archive/id/<draft>-<rev>.txt``
by default, injectable ``fetch`` for tests / offline mirrors) and diffed with difflib -- unified
text, markdown (fenced ``diff`` block) or a side-by-side HTML table.  ``LocalDiffProvider`` does the
same over a directory of ``<draft>-<rev>.txt`` files.
"""
from __future__ import annotations

import dataclasses
import difflib
import re
import urllib.error
import urllib.request
from pathlib import Path
from typing import Any, Callable

_FORMATS = ("text", "markdown", "html")
_NAME = re.compile(r"^draft-[a-z0-9][a-z0-9-]*[a-z0-9]$")
_REV = re.compile(r"^\d{2}$")


@dataclasses.dataclass
class DraftDiff:
    draft_name: str
    version_a: str
    version_b: str
    format: str
    content: str
    source: str
    url: str | None = None
    metadata: dict[str, Any] | None = None

    def to_dict(self) -> dict[str, Any]:
        return dataclasses.asdict(self)


class DraftDiffProvider:
    def getdiff(self, draft_name: str, version_a: str, version_b: str) -> DraftDiff:
        raise NotImplementedError


def _check(draft_name: str, version_a: str, version_b: str) -> None:
    if not draft_name:
        raise ValueError("draft_name cannot be empty")
    if not version_a or not version_b:
        raise ValueError("version_a and version_b must be provided")


def render_diff(a: str, b: str, fmt: str, label_a: str, label_b: str) -> tuple[str, dict]:
    la, lb = a.splitlines(), b.splitlines()
    sm = difflib.SequenceMatcher(None, la, lb, autojunk=False)
    added = sum(j2 - j1 for op, _, _, j1, j2 in sm.get_opcodes() if op in ("insert", "replace"))
    removed = sum(i2 - i1 for op, i1, i2, _, _ in sm.get_opcodes() if op in ("delete", "replace"))
    stats = {"lines_added": added, "lines_removed": removed, "similarity": round(sm.ratio(), 4)}
    if fmt == "html":
        return difflib.HtmlDiff(wrapcolumn=80).make_table(la, lb, label_a, label_b, context=True), stats
    uni = "\n".join(difflib.unified_diff(la, lb, label_a, label_b, lineterm=""))
    if fmt == "markdown":
        return f"# Diff: {label_a} -> {label_b}\n\n```diff\n{uni}\n```\n", stats
    return uni, stats


class DatatrackerDiffProvider(DraftDiffProvider):
    def __init__(self, base_url: str = "https://datatracker.ietf.org", diff_format: str = "html",
                 fetch: Callable[[str], str] | None = None, timeout: float = 30.0,
                 url_template: str = "{base}/archive/id/{draft}-{rev}.txt"):
        if diff_format not in _FORMATS:
            raise ValueError(f"diff_format must be one of {_FORMATS}")
        self.base_url = base_url.rstrip("/")
        self.diff_format = diff_format
        self.timeout = timeout
        self.url_template = url_template
        self._fetch = fetch or self._http_get
        self._cache: dict[str, str] = {}

    def _http_get(self, url: str) -> str:
        try:
            with urllib.request.urlopen(url, timeout=self.timeout) as r:
                return r.read().decode("utf-8", "replace")
        except urllib.error.HTTPError as e:
            if e.code == 404:
                raise ValueError(f"not found: {url}") from e
            raise ConnectionError(f"{url}: HTTP {e.code}") from e
        except (urllib.error.URLError, OSError) as e:
            raise ConnectionError(f"{url}: {e}") from e

    def revision_url(self, draft: str, rev: str) -> str:
        return self.url_template.format(base=self.base_url, draft=draft, rev=rev)

    def _text(self, draft: str, rev: str) -> str:
        url = self.revision_url(draft, rev)
        if url not in self._cache:
            self._cache[url] = self._fetch(url)
        return self._cache[url]

    def getdiff(self, draft_name: str, version_a: str, version_b: str) -> DraftDiff:
        _check(draft_name, version_a, version_b)
        if not _NAME.match(draft_name) or not _REV.match(version_a) or not _REV.match(version_b):
            raise ValueError(f"invalid draft name / revision: {draft_name} {version_a} {version_b}")
        a, b = self._text(draft_name, version_a), self._text(draft_name, version_b)
        content, stats = render_diff(a, b, self.diff_format, f"{draft_name}-{version_a}", f"{draft_name}-{version_b}")
        url = f"{self.base_url}/doc/{draft_name}/{version_b}/?include_text=1"
        return DraftDiff(draft_name, version_a, version_b, self.diff_format, content, "datatracker", url,
                         {"source_urls": [self.revision_url(draft_name, version_a),
                                          self.revision_url(draft_name, version_b)], **stats})


class LocalDiffProvider(DatatrackerDiffProvider):
    """Diffs ``<root>/<draft>-<rev>.txt`` files (offline mirrors, tests)."""

    def __init__(self, root: str, diff_format: str = "text"):
        self.root = Path(root)

        def read(url: str) -> str:
            p = Path(url)
            if not p.exists():
                raise ValueError(f"not found: {p}")
            return p.read_text(encoding="utf-8", errors="replace")

        super().__init__(str(self.root), diff_format, fetch=read, url_template="{base}/{draft}-{rev}.txt")

    def getdiff(self, draft_name, version_a, version_b):
        d = super().getdiff(draft_name, version_a, version_b)
        d.source, d.url = "local", None
        return d


class MockDiffProvider(DraftDiffProvider):
    def __init__(self, mock_diffs: dict | None = None, default_format: str = "text"):
        self.mock_diffs: dict[tuple[str, str, str], DraftDiff] = dict(mock_diffs or {})
        self.default_format = default_format

    def add_mock_diff(self, draft_name: str, version_a: str, version_b: str, diff: DraftDiff) -> None:
        self.mock_diffs[(draft_name, version_a, version_b)] = diff

    def getdiff(self, draft_name, version_a, version_b):
        _check(draft_name, version_a, version_b)
        hit = self.mock_diffs.get((draft_name, version_a, version_b))
        if hit is not None:
            return hit
        old = f"Old content from version {version_a}"
        new = f"New content in version {version_b}"
        if self.default_format == "html":
            content = (f"<html><body><h1>{draft_name}: {version_a} &rarr; {version_b}</h1>"
                       f"<pre><del>- {old}</del>\n<ins>+ {new}</ins></pre></body></html>")
        elif self.default_format == "markdown":
            content = (f"# Mock Diff: {draft_name}\n\nChanges from version {version_a} to {version_b}\n\n"
                       f"```diff\n- {old}\n+ {new}\n```\n")
        else:
            content = f"Mock diff for {draft_name}\nVersion {version_a} -> {version_b}\n\n- {old}\n+ {new}\n"
        return DraftDiff(draft_name, version_a, version_b, self.default_format, content, "mock",
                         f"mock://{draft_name}/{version_a}..{version_b}", {"mock": True, "generated": True})


_CUSTOM_PROVIDERS: dict[str, type] = {}


def register_draft_diff_provider(name: str, provider_class: type) -> None:
    """Plug in a provider under a driver name (reference factory.py register_provider): the class
    must subclass :class:`DraftDiffProvider`; it is built with the driver config as keyword args."""
    if not (isinstance(provider_class, type) and issubclass(provider_class, DraftDiffProvider)):
        raise TypeError(f"{provider_class!r} is not a DraftDiffProvider subclass")
    key = str(name).strip().lower()
    if not key:
        raise ValueError("provider name must be non-empty")
    _CUSTOM_PROVIDERS[key] = provider_class


def create_draft_diff_provider(cfg=None, **overrides) -> DraftDiffProvider:
    name = str(getattr(cfg, "driver_name", cfg) or "mock").strip().lower()
    kw = {k: v for k, v in dict(getattr(cfg, "driver_config", {}) or {}).items() if v is not None}
    kw.update(overrides)
    if name in _CUSTOM_PROVIDERS:
        return _CUSTOM_PROVIDERS[name](**kw)
    if name == "datatracker":
        return DatatrackerDiffProvider(**{k: kw[k] for k in ("base_url", "diff_format", "fetch", "timeout") if k in kw})
    if name == "mock":
        return MockDiffProvider(kw.get("mock_diffs"), kw.get("default_format", "text"))
    if name == "local":
        return LocalDiffProvider(kw["root"], kw.get("diff_format", "text"))
    raise ValueError(f"Unknown provider driver: {name}.")
