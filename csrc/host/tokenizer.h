// Native tokenizer runtime (host C++): word-level, WordPiece (BERT/MiniLM/MPNet), byte-level BPE
// (GPT-2/OPT) and SentencePiece-style BPE with byte fallback (Llama/Mistral), i.e. the model
// families the pipeline serves. The reference relies on HF's Rust `tokenizers` through
// AutoTokenizer (reinforcement_learning_optimization_after_rag.py:24,36,46,141,196); here the
// vocab/merges are parsed from tokenizer.json in Python and the encode/decode hot loop is C++,
// with batch encode parallelised over std::threads.
#pragma once
#include <torch/extension.h>

namespace ragtl {
void bind_tokenizer(pybind11::module& m);
}
