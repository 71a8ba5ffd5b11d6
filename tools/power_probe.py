"""Probe: amdsmi power / gfx clock readings of the visible GPU (diagnostic)."""
import time
import amdsmi

amdsmi.amdsmi_init()
hs = amdsmi.amdsmi_get_processor_handles()
print("handles", len(hs))
for h in hs:
    try:
        print("bdf", amdsmi.amdsmi_get_gpu_device_bdf(h))
    except Exception as e:
        print("bdf err", e)
    t = time.perf_counter()
    try:
        print("power", amdsmi.amdsmi_get_power_info(h))
    except Exception as e:
        print("power err", e)
    try:
        print("clk", amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX))
    except Exception as e:
        print("clk err", e)
    print("query ms %.2f" % ((time.perf_counter() - t) * 1e3))
import torch
p = torch.cuda.get_device_properties(0)
print("torch pci", getattr(p, "pci_bus_id", None), getattr(p, "pci_device_id", None), getattr(p, "pci_domain_id", None))
amdsmi.amdsmi_shut_down()
