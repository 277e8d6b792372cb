"""Host system information (reference: gopsutil/systeminfo.go:30-241, used by
diagnostics and /info)."""
from __future__ import annotations

import os
import platform
import socket
import time


class SystemInfo:
    """Uptime, platform, CPU and memory facts of this host (psutil when
    available, /proc otherwise)."""

    def __init__(self):
        try:
            import psutil  # noqa: F401
            self._ps = psutil
        except ImportError:  # pragma: no cover
            self._ps = None

    def uptime(self) -> int:
        if self._ps is not None:
            return int(time.time() - self._ps.boot_time())
        with open("/proc/uptime") as fh:
            return int(float(fh.read().split()[0]))

    def platform(self) -> str:
        return platform.system().lower()

    def family(self) -> str:
        try:
            with open("/etc/os-release") as fh:
                for line in fh:
                    if line.startswith("ID="):
                        return line.split("=", 1)[1].strip().strip('"')
        except OSError:
            pass
        return ""

    def os_version(self) -> str:
        return platform.release()

    def kernel_version(self) -> str:
        return platform.version()

    def hostname(self) -> str:
        return socket.gethostname()

    def cpu_model(self) -> str:
        try:
            with open("/proc/cpuinfo") as fh:
                for line in fh:
                    if line.startswith("model name"):
                        return line.split(":", 1)[1].strip()
        except OSError:
            pass
        return platform.processor()

    def cpu_cores(self) -> int:
        if self._ps is not None:
            return self._ps.cpu_count(logical=False) or os.cpu_count() or 0
        return os.cpu_count() or 0

    def cpu_threads(self) -> int:
        return os.cpu_count() or 0

    def cpu_mhz(self) -> int:
        if self._ps is not None:
            f = self._ps.cpu_freq()
            return int(f.current) if f else 0
        return 0

    def mem_total(self) -> int:
        if self._ps is not None:
            return int(self._ps.virtual_memory().total)
        with open("/proc/meminfo") as fh:
            for line in fh:
                if line.startswith("MemTotal:"):
                    return int(line.split()[1]) * 1024
        return 0

    def mem_used(self) -> int:
        if self._ps is not None:
            return int(self._ps.virtual_memory().used)
        return 0

    def mem_free(self) -> int:
        if self._ps is not None:
            return int(self._ps.virtual_memory().free)
        with open("/proc/meminfo") as fh:
            for line in fh:
                if line.startswith("MemFree:"):
                    return int(line.split()[1]) * 1024
        return 0

    def cpu_arch(self) -> str:
        return platform.machine()

    def gpus(self) -> list:
        """Visible GPUs (name, HBM bytes) without initialising HIP in a
        process that has not touched the GPU yet."""
        try:
            import torch
            if not torch.cuda.is_available():
                return []
            out = []
            for i in range(torch.cuda.device_count()):
                p = torch.cuda.get_device_properties(i)
                out.append({"name": p.name, "arch": getattr(p, "gcnArchName", ""), "hbmBytes": int(p.total_memory)})
            return out
        except Exception:  # noqa: BLE001
            return []

    def to_dict(self) -> dict:
        return {"hostname": self.hostname(), "platform": self.platform(), "family": self.family(),
                "osVersion": self.os_version(), "kernelVersion": self.kernel_version(), "cpuModel": self.cpu_model(),
                "cpuPhysicalCores": self.cpu_cores(), "cpuLogicalCores": self.cpu_threads(),
                "cpuMHz": self.cpu_mhz(), "cpuArch": self.cpu_arch(), "memory": self.mem_total(),
                "memoryUsed": self.mem_used(), "memoryFree": self.mem_free(),
                "uptime": self.uptime()}
