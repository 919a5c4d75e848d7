"""Event transport: publisher/subscriber API + drivers (inproc, noop, cfcbroker, rabbitmq) + validation.

Factories mirror create_publisher / create_subscriber (adapters/copilot_message_bus/
copilot_message_bus/factory.py:94,147): the validating decorator wraps the driver by default.
"""
from __future__ import annotations

from .base import EventPublisher, EventSubscriber, topic_matches
from .inproc import (CountingPublisher, InProcBroker, InProcPublisher, InProcSubscriber, NoopPublisher, NoopSubscriber,
                     default_broker, reset_default_broker)
from .validating import EventValidationError, ValidatingEventPublisher, ValidatingEventSubscriber

__all__ = ["CountingPublisher", "EventPublisher", "EventSubscriber", "topic_matches", "InProcBroker", "InProcPublisher",
           "InProcSubscriber", "NoopPublisher", "NoopSubscriber", "default_broker", "reset_default_broker",
           "EventValidationError", "ValidatingEventPublisher", "ValidatingEventSubscriber", "create_publisher",
           "create_subscriber"]


def _driver(cfg):
    if cfg is None:
        return "inproc", {}
    if isinstance(cfg, str):
        return cfg.strip().lower(), {}
    return str(cfg.driver_name).strip().lower(), dict(cfg.driver_config)


def create_publisher(cfg=None, enable_validation: bool = True, broker: InProcBroker | None = None,
                     schema_provider=None) -> EventPublisher:
    name, kw = _driver(cfg)
    if name == "inproc":
        pub = InProcPublisher(broker=broker, **kw)
    elif name == "noop":
        pub = NoopPublisher()
    elif name == "cfcbroker":
        from .cfcbroker import CfcBrokerPublisher
        pub = CfcBrokerPublisher(**kw)
    elif name == "rabbitmq":
        from .rabbitmq import RabbitMQPublisher
        pub = RabbitMQPublisher(**kw)
    elif name in ("azure_service_bus", "azureservicebus"):
        from ..cloud.azure import AzureServiceBusPublisher
        pub = AzureServiceBusPublisher(**kw)
    else:
        raise ValueError(f"unknown message_bus driver {name!r}")
    return ValidatingEventPublisher(pub, schema_provider) if enable_validation else pub


def create_subscriber(cfg=None, enable_validation: bool = True, broker: InProcBroker | None = None,
                      queue_name: str | None = None, schema_provider=None) -> EventSubscriber:
    name, kw = _driver(cfg)
    if queue_name:
        kw["queue_name"] = queue_name
    if name == "inproc":
        sub = InProcSubscriber(broker=broker, **kw)
    elif name == "noop":
        sub = NoopSubscriber()
    elif name == "cfcbroker":
        from .cfcbroker import CfcBrokerSubscriber
        sub = CfcBrokerSubscriber(**kw)
    elif name == "rabbitmq":
        from .rabbitmq import RabbitMQSubscriber
        sub = RabbitMQSubscriber(**kw)
    elif name in ("azure_service_bus", "azureservicebus"):
        from ..cloud.azure import AzureServiceBusSubscriber
        sub = AzureServiceBusSubscriber(**kw)
    else:
        raise ValueError(f"unknown message_bus driver {name!r}")
    return ValidatingEventSubscriber(sub, schema_provider) if enable_validation else sub
