"""Print HIP device properties relevant to the kernels (LDS limits, CU count)."""
import ctypes as C

hip = C.CDLL("libamdhip64.so")
attrs = {
    "MaxSharedMemoryPerBlock": 74, "SharedMemPerBlockOptin": None, "MaxSharedMemoryPerMultiprocessor": 75,
    "MultiprocessorCount": 63, "ClockRate": 59, "MemoryClockRate": 66, "MemoryBusWidth": 67, "L2CacheSize": 68,
}
# resolve enum values from the header instead of guessing
import re
hdr = open("/opt/rocm/include/hip/hip_runtime_api.h").read()
enum = {}
m = re.search(r"typedef enum hipDeviceAttribute_t \{(.*?)\} hipDeviceAttribute_t;", hdr, re.S)
val = 0
for line in m.group(1).splitlines():
    line = line.split("//")[0].strip().rstrip(",")
    if not line or line.startswith("/*") or line.startswith("*"):
        continue
    mm = re.match(r"(hipDeviceAttribute\w+)\s*(=\s*(.+))?$", line)
    if not mm:
        continue
    if mm.group(3):
        try:
            val = int(mm.group(3), 0)
        except ValueError:
            val = enum.get(mm.group(3).strip(), val)
    enum[mm.group(1)] = val
    val += 1
for name in ["hipDeviceAttributeMaxSharedMemoryPerBlock", "hipDeviceAttributeSharedMemPerBlockOptin",
             "hipDeviceAttributeMaxSharedMemoryPerMultiprocessor", "hipDeviceAttributeMultiprocessorCount",
             "hipDeviceAttributeClockRate", "hipDeviceAttributeL2CacheSize", "hipDeviceAttributeWarpSize"]:
    if name in enum:
        v = C.c_int()
        r = hip.hipDeviceGetAttribute(C.byref(v), enum[name], 0)
        print(name, r, v.value)
