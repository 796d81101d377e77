import datetime, faulthandler, hashlib, json, os, sys, time
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(ROOT, "stark-pure-rust_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
faulthandler.dump_traceback_later(60, exit=True)
import torch, torch.distributed as dist
os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = "29533"
dist.init_process_group("gloo", rank=0, world_size=1, timeout=datetime.timedelta(seconds=60))
import stark_amd as S
from stark_amd.dprove import DistCircuit, GpuProverOps, prove_distributed
torch.cuda.set_device(0)
ctx = S.Context(0)
FIX = os.path.join(ROOT, "tests", "golden", "r1cs")
r1 = open(os.path.join(FIX, "pedersen_test.r1cs"), "rb").read(); wt = open(os.path.join(FIX, "pedersen_test.wtns"), "rb").read()
golden = json.load(open(os.path.join(ROOT, "tests", "golden", "r1cs_proofs.json")))["pedersen_test"]["json_sha256"]
circ = DistCircuit(ctx, r1); print("circuit ok", flush=True)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
for i, (stream, prepared) in enumerate([(sa, True), (sb, True), (sa, False), (None, True), (sb, False)]):
    t0 = time.time()
    with torch.cuda.stream(stream if stream is not None else torch.cuda.default_stream()):
        js = prove_distributed(GpuProverOps(ctx), None if prepared else r1, wt, fri_tail_log=12, circuit=circ if prepared else None)
    print(i, stream is None, prepared, hashlib.sha256(js.encode()).hexdigest() == golden, round(time.time()-t0,3), flush=True)
