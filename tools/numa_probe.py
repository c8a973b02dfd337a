"""Where the GPU and the host threads sit: the GPU's PCI bus id and NUMA node, the process's
allowed CPUs, each NUMA node's CPUs, and the CPU the main thread runs on.  Diagnostic only."""
import ctypes
import os


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    hip.hipDeviceGetPCIBusId(buf, 64, 0)
    bus = buf.value.decode().lower()
    node = open(f"/sys/bus/pci/devices/{bus}/numa_node").read().strip() if os.path.exists(
        f"/sys/bus/pci/devices/{bus}/numa_node") else "?"
    print("gpu pci", bus, "numa node", node)
    allowed = sorted(os.sched_getaffinity(0))
    print("allowed cpus", len(allowed), allowed[:8], "...", allowed[-8:])
    base = "/sys/devices/system/node"
    for n in sorted(d for d in os.listdir(base) if d.startswith("node")):
        print(n, open(f"{base}/{n}/cpulist").read().strip())
    with open("/proc/thread-self/stat") as f:
        print("main thread on cpu", f.read().rsplit(")", 1)[1].split()[36])


if __name__ == "__main__":
    main()
