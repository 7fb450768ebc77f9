"""ASGI entry point: ``uvicorn financial_chatbot_llm_amd.serving.main:app --port 8000``.

Equivalent of the reference's ``gunicorn main:app`` (README.md:25), but run as ONE process
per GPU engine replica (the engine must not be duplicated per HTTP worker).
"""
from .app import create_app
from .factory import build_services_from_env

app = create_app(build_services_from_env())
