"""Serving fronts: the HIP LLM engine behind the llama.cpp / Ollama / OpenAI HTTP APIs, and the
HIP encoder behind the OpenAI / Ollama / text-embeddings-inference embedding APIs."""
from .embed_server import EmbedBatcher, create_embedding_app
from .llm_server import BatchScheduler, GenRequest, build_from_config, chat_prompt, create_llm_app

__all__ = ["BatchScheduler", "EmbedBatcher", "GenRequest", "build_from_config", "chat_prompt", "create_embedding_app",
           "create_llm_app"]
