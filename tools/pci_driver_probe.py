#!/usr/bin/env python3
"""Could the cold SR-IOV scan find AMD functions without the procfs device
table?  Lists every /sys/bus/pci/drivers/* directory (bound functions), reads
the vendor of the unbound rest, and times both against one read of
/proc/bus/pci/devices.  Output: profiles/pci_driver_probe_r3.txt.

    python tools/pci_driver_probe.py
"""
import os, time, collections
t0=time.perf_counter()
drivers=os.listdir('/sys/bus/pci/drivers')
bound={}
for d in drivers:
    try:
        for e in os.listdir(f'/sys/bus/pci/drivers/{d}'):
            if e.count(':')==2: bound[e]=d
    except OSError: pass
t1=time.perf_counter()
devs=os.listdir('/sys/bus/pci/devices')
t2=time.perf_counter()
unbound=[x for x in devs if x not in bound]
vend=collections.Counter()
for x in unbound:
    vend[open(f'/sys/bus/pci/devices/{x}/vendor').read().strip()]+=1
t3=time.perf_counter()
with open('/proc/bus/pci/devices','rb') as f: data=f.read()
t4=time.perf_counter()
print(f"drivers={len(drivers)} listing_ms={(t1-t0)*1e3:.3f} devices={len(devs)} bound={len(bound)} unbound={len(unbound)} vendors_unbound={dict(vend)} unbound_reads_ms={(t3-t2)*1e3:.3f} proc_table_ms={(t4-t3)*1e3:.3f}")
print(collections.Counter(bound.values()).most_common())
