"""One rank of the RCCL bootstrap smoke: gloo control plane from TF_CONFIG, then the
native RCCL communicator (unique-id broadcast + ncclCommInitRank).  Without a HIP
device the construction stops at hipSetDevice -- after the id exchange -- and the
rank reports that; with devices it reports RCCL's own rank count."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from distributed_amd.parallel import communicator as cm  # noqa: E402
from distributed_amd.parallel import runtime  # noqa: E402

rt = runtime.init()
c = cm.RcclCommunicator.__new__(cm.RcclCommunicator)
out = {"rank": rt.rank, "world": rt.world_size}
try:
    cm.RcclCommunicator.__init__(c, rt.world_size, rt.rank, rt.rank)
    out["status"] = "constructed"
    out["comm_count"] = c.native.comm_count
except Exception as e:  # no HIP device here
    out["status"] = "error"
    out["error"] = str(e)
out["uid"] = c.uid.hex() if getattr(c, "uid", None) else None
with open(os.path.join(os.environ["DAMD_TEST_OUT"], f"rccl{rt.rank}.json"), "w") as f:
    json.dump(out, f)
runtime.shutdown()
