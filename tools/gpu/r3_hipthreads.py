"""Which setup step creates the busy unnamed (HIP runtime) thread of a serving process: after
each step, list threads that used > 5 % of a core over the next second."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def busy(tag):
    def snap():
        out = {}
        for t in os.listdir("/proc/self/task"):
            try:
                st = open(f"/proc/self/task/{t}/stat").read()
            except OSError:
                continue
            rp = st.rindex(")")
            name = st[st.index("(") + 1:rp]
            f = st[rp + 2:].split()
            out[t] = (name, int(f[11]) + int(f[12]))
        return out
    a = snap()
    time.sleep(1.0)
    b = snap()
    hot = {t: (b[t][0], b[t][1] - a[t][1]) for t in b if t in a and b[t][1] - a[t][1] > 5}
    print(f"{tag}: {len(b)} threads, busy: {hot}", flush=True)


busy("start")
import torch  # noqa: E402
busy("import torch")
torch.cuda.init()
x = torch.ones(4, device="cuda")
busy("cuda init")
from gale._native import native  # noqa: E402
from gale.config import GaleConfig  # noqa: E402
from gale.engine import Engine  # noqa: E402
busy("import gale")
cfg = GaleConfig(topology_name="t", input_topic="in", output_topic="out", model="resnet20",
                 replicas=1, gpu_ingest=False).validate()
from gale.models import get_model  # noqa: E402
from gale.parallel.weights import materialize_weights  # noqa: E402
from gale.runtime.replica import ModelReplica  # noqa: E402
net = get_model("resnet20")
packed = materialize_weights(net, torch.device("cuda", 0))
busy("weights")
rep = ModelReplica(net, packed, max_batch=256, slots=3)
busy("replica")
rep.capture()
busy("graph capture")
K = native().kafka
b = K.Broker()
b.start()
b.create_topic("in", 1)
b.create_topic("out", 1)
cfg.bootstrap = f"127.0.0.1:{b.port}"
eng = Engine(cfg, devices=[0], model_replicas=[rep])
busy("engine (GpuReplica)")
eng._native.enable_gpu_ingest(0, 2, 20)
busy("gpu ingest")
eng.start()
busy("engine started (idle)")
eng.stop()
b.stop()
busy("stopped")
