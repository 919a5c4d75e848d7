"""Serving fronts: the HIP LLM engine behind the llama.cpp / Ollama / OpenAI HTTP APIs."""
from .llm_server import BatchScheduler, GenRequest, build_from_config, chat_prompt, create_llm_app

__all__ = ["BatchScheduler", "GenRequest", "build_from_config", "chat_prompt", "create_llm_app"]
