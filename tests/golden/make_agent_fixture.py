#!/usr/bin/env python3
"""Fixture generator (run in the build container, where /root/reference exists):

* the actor of the shipped PPO agent ``ppo_agents/PFCA_see_3_obs_17_90.zip`` -- its ``policy.pth``
  is a plain torch state_dict, read with ``torch.load(weights_only=True)`` (no unpickling of code);
  only the policy MLP (27-64-64-2, tanh), ``action_net`` and ``log_std`` are kept, as float32 npz;
* the reference's own closed-loop results for that agent
  (``best_models_config_and_res/run17see3/res/<scenario>/results.txt``, 100 runs each) and its
  env config (``env_train_config.txt`` is a Python dict literal: parsed with ast.literal_eval).

* the per-episode arrays the reference saved beside each results.txt (collisions / rewards / apes /
  time_spent ``.npy``, read with ``numpy.load(allow_pickle=False)``) and the results.txt text itself,
  so the harness's results writer can be checked byte for byte against the reference's output.

Outputs: tests/golden/agent_17_90.npz, tests/golden/agent_17_90_results.json,
tests/golden/agent_17_90_episodes.npz.
"""
import ast
import io
import json
import os
import zipfile

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
AGENT = "ppo_agents/PFCA_see_3_obs_17_90.zip"
RUN = "best_models_config_and_res/run17see3"


def main():
    z = zipfile.ZipFile(os.path.join(REF, AGENT))
    sd = torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True, map_location="cpu")
    keep = ["mlp_extractor.policy_net.0.weight", "mlp_extractor.policy_net.0.bias",
            "mlp_extractor.policy_net.2.weight", "mlp_extractor.policy_net.2.bias",
            "action_net.weight", "action_net.bias", "log_std"]
    np.savez(os.path.join(HERE, "agent_17_90.npz"),
             **{k.replace(".", "_"): sd[k].numpy().astype(np.float32) for k in keep})
    res, txt, eps = {}, {}, {}
    resdir = os.path.join(REF, RUN, "res")
    for scn in sorted(os.listdir(resdir)):
        f = os.path.join(resdir, scn, "results.txt")
        if not os.path.exists(f):
            continue
        d = {}
        for line in open(f):
            k, _, v = line.partition(":")
            v = v.strip()
            try:
                d[k.strip()] = float(v)
            except ValueError:
                d[k.strip()] = v
        res[scn] = d
        txt[scn] = open(f).read()
        for k in ("collisions", "rewards", "apes", "time_spent"):
            eps[f"{scn}__{k}"] = np.load(os.path.join(resdir, scn, f"{k}.npy"), allow_pickle=False)
    cfg = ast.literal_eval(open(os.path.join(REF, RUN, "env_train_config.txt")).read())
    np.savez(os.path.join(HERE, "agent_17_90_episodes.npz"), **eps)
    json.dump({"agent": AGENT, "source": RUN + "/res/*/results.txt", "env_config": cfg, "results": res,
               "results_txt": txt},
              open(os.path.join(HERE, "agent_17_90_results.json"), "w"), indent=1, default=str)
    print("wrote", len(res), "scenario results")


if __name__ == "__main__":
    main()
