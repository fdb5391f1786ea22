"""Print what parallel/topology.py sees on this host (GPU box diagnostics)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.parallel import topology  # noqa: E402

print("env", {k: os.environ.get(k) for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                                            "OMP_NUM_THREADS")})
aff = sorted(os.sched_getaffinity(0))
print("affinity", len(aff), topology.compress(aff))
print("cpu.max quota", topology.cpu_quota(), "cpu_count", os.cpu_count())
print("gpus", [g.__dict__ for g in topology.gpus()])
print("numa", {k: topology.compress(v) for k, v in topology.numa_cpus().items()})
for n in (1, 2, 4, 8):
    print("plan", n, json.dumps([p.as_dict() for p in topology.plan(n)]))
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch
    p = torch.cuda.get_device_properties(0)
    print("torch", {k: getattr(p, k, None) for k in ("name", "pci_bus_id", "pci_device_id", "pci_domain_id",
                                                     "multi_processor_count", "gcnArchName")})
