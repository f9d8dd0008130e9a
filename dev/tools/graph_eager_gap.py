"""Graph vs eager fold loop at a small learning rate (tests/test_model_classifier.py
test_model_graph_training_tracks_eager): the per-step relative loss gap, repeated."""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_model_classifier import CLS  # noqa: E402
from tensorflowdistributedlearning_amd.model import Model  # noqa: E402

for rep in range(int(os.environ.get("REPS", "3"))):
    with tempfile.TemporaryDirectory() as d:
        kw = dict(CLS, device=None, save_checkpoints_steps=100, save_best=0, lr=0.002, momentum=0.0)
        ra = Model(d + "/e", "", hip_graph="off", **kw).train(192, None, 16, 4)[0]
        rb = Model(d + "/g", "", **kw).train(192, None, 16, 4)[0]
        ea = Model(d + "/e2", "", hip_graph="off", **kw).train(192, None, 16, 4)[0]
        g = np.abs(np.array(rb["train_loss"]) - ra["train_loss"]) / np.array(ra["train_loss"])
        e = np.abs(np.array(ea["train_loss"]) - ra["train_loss"]) / np.array(ra["train_loss"])
        print("graph-vs-eager", np.round(g, 4), " eager-vs-eager", np.round(e, 4), flush=True)
