"""RAG core: reference prompt template, answer extraction, retrieve-then-generate pipeline."""
from .prompt import INSTRUCTION, build_prompt, extract_answer, fit_docs  # noqa: F401
from .pipeline import RagAnswer, RagPipeline  # noqa: F401
