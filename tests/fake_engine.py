"""CPU stand-in for LLMEngine used by the EngineGroup tests (worker factory target): deterministic
per-candidate token streams derived from (seed, candidate index), optional per-step delay."""
import time


class _Seq:
    def __init__(self, g, index, seed):
        self.group, self.index, self.seed = g, index, seed
        self.tokens, self.finished = [], False


class _Group:
    def __init__(self, params, n, cb):
        base = params.seed or 0
        self.params, self.callback = params, cb
        self.seqs = [_Seq(self, i, base * 1000003 + params.seed_offset + i) for i in range(n)]

    @property
    def finished(self):
        return all(s.finished for s in self.seqs)


class _Ev:
    def __init__(self, seq, tid):
        self.seq, self.token_id, self.text = seq, tid, chr(97 + tid % 26)
        self.logprob, self.top_logprobs = -0.5, [(tid, -0.5)]
        self.finished, self.finish_reason = False, None


class FakeEngine:
    def __init__(self, delay, log=None):
        self.groups, self.delay = [], delay
        self.running, self.waiting = [], []
        self.log = log  # tensor-parallel tests: one line per step (the batch each rank stepped)

    def add_request(self, prompt, params, n=1, callback=None):
        g = _Group(params, n, callback)
        self.groups.append(g)
        return g

    def has_work(self):
        return any(not g.finished for g in self.groups)

    def step(self):
        time.sleep(self.delay)
        for g in self.groups:
            for s in g.seqs:
                if s.finished:
                    continue
                tid = (s.seed + len(s.tokens)) % 1000
                s.tokens.append(tid)
                ev = _Ev(s, tid)
                if len(s.tokens) >= g.params.max_tokens:
                    s.finished, ev.finished, ev.finish_reason = True, True, "length"
                if g.callback is not None:  # tensor-parallel followers stream nothing
                    g.callback(ev)
        self.groups = [g for g in self.groups if not g.finished]
        if self.log is not None:
            self.log.write(" ".join(f"{s.seed}:{len(s.tokens)}" for g in self.groups for s in g.seqs) + "\n")
            self.log.flush()

    def abort(self, g):
        for s in g.seqs:
            s.finished = True

    def fail_all(self, msg):
        out = [g for g in self.groups if not g.finished]
        for g in out:
            self.abort(g)
        return out


def make(spec, wid):
    log = None
    if spec.get("log_dir"):
        log = open(f"{spec['log_dir']}/w{wid}_rank{int(spec.get('tp_rank', 0))}.log", "w")
    return FakeEngine(float(spec.get("delay", 0.0)), log)
