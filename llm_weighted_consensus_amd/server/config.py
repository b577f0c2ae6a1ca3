"""Server configuration from the environment (+ optional `.env`).

Every variable of the reference (src/main.rs:3-37) keeps its name and default; the remote provider
bases are OPTIONAL here (they become the fallback tier behind the local MI355X engine).  New
variables configure the local engine:

  LWC_MODELS        JSON {name: {"arch": "llama-3-8b", "weights": "random:<seed>" | <path>,
                          "max_model_len": 4096, "max_batch": 512, "fp8": false, "tp": 1}}   (default: none)
                    "tp": T (MoE decoders, BASELINE config 5) serves each replica tensor-parallel over T
                    consecutive LWC_GPUS entries — one process per GPU, the IPC one-shot all-reduce (C3)
                    inside every forward, the ranks stepping in lockstep behind the replica's rank 0
  LWC_EMBED_MODELS  JSON {name: {"arch": "bge-large-en-v1.5", "weights": "random:<seed>" | <path>}}
  LWC_GPU           device index for this process's engine (one process per GPU)
  LWC_GPUS          comma list of devices: serve each model through an EngineGroup (one worker process
                    per listed GPU, candidates of a request split across them, failover; "0" = one worker)
  LWC_DEVICE        "cuda" (default) or "cpu": CPU runs embedding models only, on the fp32 reference
                    path (BASELINE config 1: canned completions + bge-small cosine consensus, no GPU)
  LWC_KV_FRACTION   fraction of free HBM given to the paged KV cache (default 0.85)
  LWC_ARCHIVE_PATH  append-only JSONL log of completions (checkpoint/resume of the archive)
  LWC_REGISTRY_PATH JSON file persisting registered score models
  LWC_CHUNKED_PREFILL prompt tokens per engine step (default 2048): each step is ONE forward over every
                    running sequence's next token and up to this many prompt tokens (mixed chunked prefill,
                    paged-KV prefill attention); 0 = whole admission batches before decoding.  4096 trades
                    p99 for throughput (profiles/serve_load.md)
  LWC_TRAINING_TABLE_PATH  append-only JSONL of training-table rows (learned voter weights), replayed on start
  LWC_FAULT         fault injection for tests: worker_crash | slow_decode | bad_logprobs | oom
  LWC_CONSTRAINED_LOGPROBS  1: constrained (json_schema / tool-call) voters get logprobs over the allowed
                    tokens, so a key letter's vote is the exact restricted softmax over its siblings
                    instead of whatever of them made the raw top-k (default 0 = reference semantics)
  LWC_KV_RESERVE_TOKENS  generation tokens reserved per sequence at admission (default 256; "none" = the
                    whole max_tokens, no preemption): longer generations draw on the shared pool and the
                    youngest requests are preempted by swapping their KV to host memory when it runs dry
  LWC_REQUEST_TIMEOUT_MS  default request deadline (an x-timeout-ms header overrides it per request; the
                    engine drops or aborts a request past its deadline); x-priority orders admission
  LWC_SHARD_VOTERS  1: voter-sharded deployment — one server process per GPU under torchrun / a
                    launcher (RANK / WORLD_SIZE / LOCAL_RANK); rank 0 serves HTTP, resolves each score
                    request once and sends every live follower its share of the voters over a TCP link
                    (voter i -> live[i % len(live)]); followers stream every voter chunk back as it is
                    produced and rank 0 merges them live and tallies (C2, score/sharded.py,
                    parallel/shard_link.py)
  LWC_SHARD_HB_S    follower heartbeat period on the shard links (default 0.5 s)
  LWC_SHARD_DEAD_S  silence after which a follower counts as dead (default 10 s; a closed socket — a
                    follower process that exited — counts at once): its unfinished voters become error
                    choices and later requests run on the survivors
  LWC_SHARD_LINK_HOST  interface the leader's link listener binds (default loopback: one node)
  LWC_SHARD_LINK_FILE  the leader writes its link address + secret here (mode 0600); a follower restarted
                    outside the bring-up group (LWC_SHARD_REJOIN_RANK=<rank>) authenticates with it and is
                    re-admitted: live ranks return to full size and later requests give it voters again
  LWC_SHARD_WAIT_S  bound on a request's wait for its followers when it carries no deadline (default 300 s;
                    with a deadline: the deadline plus LWC_SHARD_GRACE_S, default 5 s)
  LWC_GPU_TALLY     N >= 1: tallies of score requests finishing in the same event-loop turn are batched,
                    and batches of at least N run as one vote_tally launch (K10b) on this process's GPU
                    (launched and read back on a worker thread); default 2 when this process runs an
                    engine on its GPU (measured +10.8 % req/s, profiles/serve_load.md), else off; 0: the
                    host C++ tally per request
  LWC_RESPAWN       1 (default): an EngineGroup worker (or a whole TP replica) that dies is replaced by a fresh
                    child process with exponential backoff (LWC_RESPAWN_BACKOFF_S, default 0.5 s, doubling to
                    30 s), at most LWC_MAX_RESPAWNS times per worker (default 8); 0: a dead worker stays dead
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional


def _load_dotenv(path: str = ".env") -> None:
    if not os.path.exists(path):
        return
    with open(path, "r", encoding="utf-8") as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#") or "=" not in line:
                continue
            k, v = line.split("=", 1)
            os.environ.setdefault(k.strip(), v.strip().strip('"').strip("'"))


@dataclass
class Config:
    backoff_current_interval_millis: int = 100
    backoff_initial_interval_millis: int = 100
    backoff_randomization_factor: float = 0.5
    backoff_multiplier: float = 1.5
    backoff_max_interval_millis: int = 1000
    backoff_max_elapsed_time_millis: int = 40000
    first_chunk_timeout_millis: int = 10000
    other_chunk_timeout_millis: int = 60000
    openai_api_base: Optional[str] = None
    openai_api_key: Optional[str] = None
    openai_apis: Optional[str] = None
    openai_user_agent: Optional[str] = None
    openai_x_title: Optional[str] = None
    openai_referer: Optional[str] = None
    address: str = "0.0.0.0"
    port: int = 5000
    # local engine
    models: Dict[str, dict] = field(default_factory=dict)
    embed_models: Dict[str, dict] = field(default_factory=dict)
    gpu: int = 0
    gpus: List[int] = field(default_factory=list)
    device: str = "cuda"
    constrained_logprobs: bool = False
    prefix_caching: bool = True
    chunked_prefill: int = 2048
    kv_fraction: float = 0.85
    archive_path: Optional[str] = None
    training_table_path: Optional[str] = None
    registry_path: Optional[str] = None
    fault: Optional[str] = None
    shard_voters: bool = False
    kv_reserve_tokens: Optional[int] = 256
    request_timeout_ms: Optional[int] = None
    gpu_tally: Optional[str] = None
    respawn: bool = True
    max_respawns: int = 8
    respawn_backoff_s: float = 0.5

    @classmethod
    def from_env(cls, dotenv: bool = True) -> "Config":
        if dotenv:
            _load_dotenv()
        e = os.environ
        c = cls()
        ints = ["backoff_current_interval_millis", "backoff_initial_interval_millis", "backoff_max_interval_millis",
                "backoff_max_elapsed_time_millis", "first_chunk_timeout_millis", "other_chunk_timeout_millis", "port"]
        floats = ["backoff_randomization_factor", "backoff_multiplier"]
        strs = ["openai_api_base", "openai_api_key", "openai_apis", "openai_user_agent", "openai_x_title",
                "openai_referer", "address"]
        for k in ints:
            if k.upper() in e:
                setattr(c, k, int(e[k.upper()]))
        for k in floats:
            if k.upper() in e:
                setattr(c, k, float(e[k.upper()]))
        for k in strs:
            if k.upper() in e:
                setattr(c, k, e[k.upper()])
        if "LWC_MODELS" in e:
            c.models = json.loads(e["LWC_MODELS"])
        if "LWC_EMBED_MODELS" in e:
            c.embed_models = json.loads(e["LWC_EMBED_MODELS"])
        c.gpu = int(e.get("LWC_GPU", e.get("LOCAL_RANK", "0")))
        c.device = e.get("LWC_DEVICE", "cuda").lower()
        c.constrained_logprobs = e.get("LWC_CONSTRAINED_LOGPROBS", "0") == "1"
        c.prefix_caching = e.get("LWC_PREFIX_CACHE", "1") == "1"
        c.chunked_prefill = int(e.get("LWC_CHUNKED_PREFILL", "2048"))
        if e.get("LWC_GPUS"):
            c.gpus = [int(x) for x in e["LWC_GPUS"].split(",") if x.strip()]
        c.kv_fraction = float(e.get("LWC_KV_FRACTION", "0.85"))
        c.archive_path = e.get("LWC_ARCHIVE_PATH")
        c.registry_path = e.get("LWC_REGISTRY_PATH")
        c.training_table_path = e.get("LWC_TRAINING_TABLE_PATH")
        c.fault = e.get("LWC_FAULT")
        c.shard_voters = e.get("LWC_SHARD_VOTERS", "0") == "1"
        c.gpu_tally = e.get("LWC_GPU_TALLY")
        c.respawn = e.get("LWC_RESPAWN", "1") == "1"
        c.max_respawns = int(e.get("LWC_MAX_RESPAWNS", "8"))
        c.respawn_backoff_s = float(e.get("LWC_RESPAWN_BACKOFF_S", "0.5"))
        if "LWC_KV_RESERVE_TOKENS" in e:
            v = e["LWC_KV_RESERVE_TOKENS"].strip().lower()
            c.kv_reserve_tokens = None if v in ("", "none", "max") else int(v)
        if e.get("LWC_REQUEST_TIMEOUT_MS"):
            c.request_timeout_ms = int(e["LWC_REQUEST_TIMEOUT_MS"])
        return c

    def api_bases(self):
        """Remote tier (reference main.rs:76-96); empty instead of a panic when unset."""
        from ..chat.remote import ApiBase

        if self.openai_apis:
            return [ApiBase(**x) for x in json.loads(self.openai_apis)]
        if self.openai_api_base and self.openai_api_key:
            return [ApiBase(self.openai_api_base, self.openai_api_key)]
        return []

    def backoff(self):
        from ..chat.remote import Backoff

        return Backoff(initial_interval=self.backoff_initial_interval_millis / 1000.0,
                       randomization_factor=self.backoff_randomization_factor, multiplier=self.backoff_multiplier,
                       max_interval=self.backoff_max_interval_millis / 1000.0,
                       max_elapsed=self.backoff_max_elapsed_time_millis / 1000.0)
