"""Writes tests/golden/unreserve_kat.json: known answers transcribed by hand from the reference's Go tests of the
Reserve / Unreserve and DeviceShare restore semantics that kg_reserve / kg_unreserve / kg_replay run on the device
(SURVEY §8a rows a10, a12, a16). Values and expected results are copied from the cited test tables; tests/
test_unreserve_kat.py builds each case on a small config-5 cluster and runs it on the oracle session and the device.
No reference source is executed or embedded.

Units: GPU core / memory-ratio in percent of a card, GPU memory in Gi; cpu in milli-cores, memory in Gi.
Minor numbering: the reference's Test_Plugin_ReservationRestore uses minors 1 and 2; here they are minors 0 and 1 of
a node with two GPUs (a minor's number enters no decision of these cases).

Not transcribed (not on the device path; the reference tests exercise the control plane there):
- TestUnreserve "unreserve reserve pod" and TestUnreserveWhenReservationDeleted (reservation/plugin_test.go:4429,4515):
  the Unreserve of a reserve pod (forgetReservation on the reservation cache); the engine does not place reserve pods.
- TestUnreserve "skip unreserve when pod is assigned to node eventually" (:4447): the reservation-allocated annotation
  after PreBind; the cache part (AssignedPods emptied) is the "unreserve pod in reservation" case.
- Test_Plugin_Unreserve's FPGA / RDMA minors (deviceshare/plugin_test.go:5265-5300): the device tables hold GPU minors.
- Test_allocateWithNominated "reserve pod without pre-allocation" and "reservation-ignored pod"
  (deviceshare/reservation_test.go:1189,1204): reserve pods and the reservation-ignored label are host-side.
"""
import json
import os

GPU_NODE = {"minors": {"0": [100, 100, 8], "1": [100, 100, 8]}}

cases = [
    # deviceshare/reservation_test.go:40-226 Test_Plugin_ReservationRestore: the reserve pod of reservation-1 holds
    # minor 1 whole (updateCacheUsed of its allocation), allocated-pod-1 of the reservation uses 50 / 4Gi / 50 of it;
    # RestoreReservation gives the matched reservation allocatable = minor 1 whole, allocated = its pod's share,
    # remained = the rest, and the same merged tables. A pod of the reservation's owners requesting 50 / 4Gi
    # (the test's podRequests) allocates from the remained part (allocateWithNominated -> tryAllocateFromReusable);
    # one requesting a whole GPU does not fit the remained part and (the reservation not required) allocates outside it.
    {"name": "Test_Plugin_ReservationRestore", "ref": "deviceshare/reservation_test.go:40-226",
     "node": GPU_NODE, "used": {"0": [150, 150, 12]},
     "reservation": {"cls": 0, "policy": "Default", "cpu_m": 1000, "mem": 1, "dev_alloc": {"0": [100, 100, 8]},
                     "dev_allocated": {"0": [50, 50, 4]}, "allocated_pods": 1},
     "want_parts": {"allocatable": {"0": [100, 100, 8]}, "allocated": {"0": [50, 50, 4]},
                    "remained": {"0": [50, 50, 4]}, "merged_matched_allocatable": {"0": [100, 100, 8]},
                    "merged_matched_allocated": {"0": [50, 50, 4]}},
     "pods": [
         {"name": "pod of the owners, 50 core / 4Gi", "cls": 0, "gpu": {"core": 50, "mem": 4},
          "want_minors": [0], "want_nominated": True, "want_rsv_allocated_after": {"0": [100, 100, 8]}},
         {"name": "pod of the owners, one whole GPU", "cls": 0, "gpu": {"core": 100, "ratio": 100},
          "want_minors": [1], "want_nominated": True},
     ]},
    # deviceshare/reservation_test.go:1126-1280 Test_allocateWithNominated "normal pod without nominated reservation":
    # allocateWithNominated returns no result (nil): the pod allocates outside every reservation, from the node's free
    # minors as the pods that match nothing see them (the reservation holding minor 0 keeps it).
    {"name": "Test_allocateWithNominated normal pod without nominated reservation",
     "ref": "deviceshare/reservation_test.go:1219-1230",
     "node": GPU_NODE, "used": {"0": [150, 150, 12]},
     "reservation": {"cls": 0, "policy": "Default", "cpu_m": 1000, "mem": 1, "dev_alloc": {"0": [100, 100, 8]},
                     "dev_allocated": {"0": [50, 50, 4]}, "allocated_pods": 1},
     "pods": [
         {"name": "normal pod", "cls": -1, "gpu": {"core": 50, "mem": 4}, "want_minors": [1], "want_nominated": False},
     ]},
    # reservation/plugin_test.go:4360-4512 TestUnreserve "unreserve pod in reservation": reservation2C4G reserves 2 cpu /
    # 4Gi, test-pod requests 2 cpu / 4Gi and is nominated to it; after Reserve + Unreserve the reservation's
    # AssignedPods is empty (forgetPods -> RemoveAssignedPod: Allocated back to zero, no assigned pod).
    {"name": "TestUnreserve unreserve pod in reservation", "ref": "reservation/plugin_test.go:4436-4441,4494-4501",
     "node": GPU_NODE, "used": {},
     "reservation": {"cls": 1, "policy": "Default", "cpu_m": 2000, "mem": 4, "allocated_pods": 0},
     "pods": [
         {"name": "test-pod", "cls": 1, "cpu_m": 2000, "mem": 4, "want_nominated": True,
          "want_info_after_reserve": {"allocated": [2000, 4], "allocated_pods": 1},
          "want_info_after_unreserve": {"allocated": [0, 0], "allocated_pods": 0}},
     ]},
    # reservation/plugin_test.go:4431-4434 TestUnreserve "node without reservations": nothing to forget.
    {"name": "TestUnreserve node without reservations", "ref": "reservation/plugin_test.go:4431-4434",
     "node": GPU_NODE, "used": {}, "reservation": None,
     "pods": [{"name": "pod", "cls": -1, "cpu_m": 1000, "mem": 1, "want_nominated": False}]},
    # deviceshare/plugin_test.go:5213-5523 Test_Plugin_Unreserve "normal case": the pod's allocation (minors 0 and 1,
    # each 100 / 100 / 16Gi) is given back (updateCacheUsed(add=false)): every minor free again, nothing used.
    {"name": "Test_Plugin_Unreserve normal case", "ref": "deviceshare/plugin_test.go:5254-5520",
     "node": {"minors": {"0": [100, 100, 16], "1": [100, 100, 16]}}, "used": {"0": [100, 100, 16], "1": [100, 100, 16]},
     "reservation": None,
     "unreserve_only": {"gpu": {"core": 100, "ratio": 100, "count": 2}, "minors": [0, 1],
                        "want_free": {"0": [100, 100, 16], "1": [100, 100, 16]}}},
    # deviceshare/plugin_test.go:5230-5251 Test_Plugin_Unreserve "return when skip == true" / "return missing
    # preFilterState": a pod without a device request gives nothing back.
    {"name": "Test_Plugin_Unreserve skip", "ref": "deviceshare/plugin_test.go:5230-5251",
     "node": {"minors": {"0": [100, 100, 16], "1": [100, 100, 16]}}, "used": {"0": [100, 100, 16], "1": [100, 100, 16]},
     "reservation": None,
     "unreserve_only": {"gpu": None, "minors": [], "want_free": {"0": [0, 0, 0], "1": [0, 0, 0]}}},
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "unreserve_kat.json")
    with open(out, "w") as f:
        json.dump(cases, f, indent=1)
    print("wrote", out, len(cases), "cases")
