import collections, sys, os, torch, importlib, math
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from rag_tl_domainllm_optimizer_amd import ops
from rag_tl_domainllm_optimizer_amd.models import build_model
from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
from rag_tl_domainllm_optimizer_amd.retrieval import Encoder
from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer
from rag_tl_domainllm_optimizer_amd.data import SyntheticCorpus
C = ops.native()
calls = collections.Counter()
phase = ["x"]
orig = C.gemm
class Wrap:
    def __getattr__(self, k): return getattr(C, k)
    def gemm(self, x, w, u=None, ub=None, bias=None, act=0, out_f32=False, out=None, residual=None, norm_eps=0.0):
        calls[(phase[0], tuple(x.shape), tuple(w.shape), u is not None, bias is not None, act, out_f32)] += 1
        return orig(x, w, u, ub, bias, act, out_f32, out, residual, norm_eps)
W = Wrap()
import rag_tl_domainllm_optimizer_amd.ops._ext as E
E._C = W
dev = torch.device("cuda")
pol = build_model("mistral-7b", device=dev, dtype=torch.bfloat16, fast_init=True)
tok = Tokenizer.synthetic(pol.cfg.vocab_size, pol.cfg.arch)
encm = build_model("minilm-l6", device=dev, dtype=torch.bfloat16, fast_init=True).eval()
enc = Encoder(encm, Tokenizer.synthetic(encm.cfg.vocab_size, encm.cfg.arch), max_length=128)
corp = SyntheticCorpus(tok.words(), n_docs=500, doc_words=48)
tr = PPOTrainer(pol, tok, RewardModel(enc), PPOConfig(max_new_tokens=128, max_prompt_tokens=320, minibatch_size=16, lora_r=16), max_batch=64)
items = corp.sample_queries(64)
batch = {"query": [i.query for i in items], "retrieved_docs": [[corp.docs[j] for j in range(k, k+3)] for k in range(64)], "ground_truth": [i.ground_truth for i in items]}
import contextlib
orig_phase = tr.timer.phase
@contextlib.contextmanager
def ph(name):
    phase[0] = name
    with orig_phase(name):
        yield
tr.timer.phase = ph
tr.step(batch)
for k, v in sorted(calls.items(), key=lambda kv: -kv[1])[:30]: print(v, k)
