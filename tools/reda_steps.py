import json, os, sys
sys.path.insert(0, '/root/repo' if os.path.exists('/root/repo') else os.environ.get('GRAFT_REPO_ROOT', '.'))
import torch
import bench
from marl_sap_amd.action_selectors.sap_selectors import SequentialAssignmentProblemSelector

log = []
orig = SequentialAssignmentProblemSelector.select_action
def wrapped(self, agent_inputs, *a, **k):
    B = agent_inputs.shape[0]
    if self.count_steps is None or self.count_steps.shape[0] != B:
        self.count_steps = torch.zeros(B, dtype=torch.int32, device=agent_inputs.device)
    first = getattr(self, "_cold_next", None)
    out = orig(self, agent_inputs, *a, **k)
    s = self.count_steps.to(torch.int64)
    fast = (s & 0xffff).sum().item(); exact = (s >> 16).sum().item(); nexact = int(((s >> 16) > 0).sum().item())
    log.append((self.calls, fast / B, exact / B, nexact))
    return out
SequentialAssignmentProblemSelector.select_action = wrapped
a = bench.parse(["--cpu-baseline", "0", "--secondary", "0", "--steps", "40"])
dev = torch.device("cuda", 0)
E = bench.CONFIGS[a.config]["envs"]
js = dict(mac="jumpstart_mac", use_rnn=False, jumpstart_action_selector="haa_selector",
          jumpstart_epsilon_start=1.0, jumpstart_epsilon_finish=0.0, jumpstart_epsilon_anneal_time=20000,
          jumpstart_evaluation_epsilon=0.0)
r = bench.run_leg(a, dev, 1, E, a.steps, 2 * a.T, selector="sap", agent="rnn", count_lsa=False, **js,
                  epsilon_start=1.0, epsilon_finish=0.0, epsilon_anneal_time=20000)
for c in log[-45:]:
    print("call %d fast_steps/env %.1f exact_steps/env %.2f envs_on_exact %d" % c)
