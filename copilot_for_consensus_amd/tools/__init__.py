"""Operational tools (the reference's scripts/ directory): stuck-document retry job,
failed-queue CLI, Prometheus exporters, Drain log mining, schema export / validation, gateway
(OpenAPI + nginx) generation.  Each module has a ``main`` and runs with ``python -m``."""
