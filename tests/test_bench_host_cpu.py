"""bench.py's host-placement helpers on the CPU: the NUMA node's CPU list parsing and the
main-thread pinning switch (the GPU-side effect is measured in profiles/r06z2_pin_cpu_ab.txt and
r06z3_numa_local_ab.txt)."""
import bench


def test_parse_cpulist():
    assert bench.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert bench.parse_cpulist("64-127,192-255") == set(range(64, 128)) | set(range(192, 256))
    assert bench.parse_cpulist("") == set()


def test_pin_off_is_a_no_op():
    assert bench.pin_main_thread("off") == "off"
    assert bench.pin_main_thread("") == "off"
