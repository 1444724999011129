import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, os, json
from dryad_amd.parallel import affinity as A
p = torch.cuda.get_device_properties(0)
addr = A.pci_address(p)
print(json.dumps({"addr": addr, "node": A.gpu_numa_node(addr), "cpus_before": len(os.sched_getaffinity(0)),
                  "bind": A.bind_to_gpu(0), "cpus_after": len(os.sched_getaffinity(0)),
                  "props": {k: getattr(p, k) for k in ("pci_bus_id", "pci_device_id", "pci_domain_id") if hasattr(p, k)}}))
