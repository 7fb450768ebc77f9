"""financial_chatbot_llm_amd -- MI355X-native RAG chat-agent serving stack.

Same capabilities as kyshu11027/financial-chatbot-llm ("Penny"): Kafka-driven tool-calling
finance agent with transaction retrieval, re-designed so the LLM, the embedding encoder and
the vector search run locally on AMD Instinct MI355X (gfx950) GPUs.

Layers (bottom-up): ``csrc`` (HIP/CDNA4 kernels + C++ runtime) -> ``ops`` (Python bindings with
fp32 reference fallbacks) -> ``models`` (Llama-3 / Mixtral / BERT) -> ``parallel`` (TP over
RCCL) -> ``engine`` (paged KV, continuous batching, hipGraph decode) -> ``retrieval`` ->
``agent`` -> ``serving`` (FastAPI + Kafka worker).
"""
__version__ = "0.1.0"
