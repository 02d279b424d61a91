/* fault_probe.c -- test infrastructure (tests/conftest.py), host code only: records the
 * details the HIP runtime does not print of a GPU memory fault in this process.
 *
 * HIP's own handler logs only "Memory Fault Error" (rocdevice.cpp, AMD_LOG_LEVEL >= 1) and
 * turns every later call into hipErrorIllegalAddress.  ROCr passes the same event -- with
 * the faulting virtual address and the reason bits -- to every system event handler a
 * process registers (hsa_amd_register_system_event_handler), so this one prints them at once
 * to stderr (pytest's capture puts the line under the test that was running) and keeps the
 * first fault for hg_fault_probe_read().  Built by __graft_entry__.build() into
 * tests/_build/libfault_probe.so; never linked into the product. */
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include <stdio.h>

static volatile int g_events;      /* memory faults and HW exceptions seen */
static volatile int g_type = -1;   /* first event's hsa_amd_event_type_t */
static volatile uint64_t g_va;     /* first memory fault's virtual address */
static volatile uint32_t g_reason; /* its hsa_amd_memory_fault_reason_t bits */

static hsa_status_t on_event(const hsa_amd_event_t* e, void* data) {
    (void)data;
    if (e->event_type == HSA_AMD_GPU_MEMORY_FAULT_EVENT) {
        const uint64_t va = e->memory_fault.virtual_address;
        const uint32_t r = e->memory_fault.fault_reason_mask;
        if (g_events++ == 0) {
            g_type = (int)e->event_type;
            g_va = va;
            g_reason = r;
        }
        fprintf(stderr,
                "fault_probe: GPU memory fault at VA 0x%016llx, reason 0x%x%s%s%s%s%s (agent 0x%llx)\n",
                (unsigned long long)va, r, (r & HSA_AMD_MEMORY_FAULT_PAGE_NOT_PRESENT) ? " page-not-present" : "",
                (r & HSA_AMD_MEMORY_FAULT_READ_ONLY) ? " write-to-read-only" : "",
                (r & HSA_AMD_MEMORY_FAULT_HOST_ONLY) ? " host-only-page" : "",
                (r & HSA_AMD_MEMORY_FAULT_IMPRECISE) ? " imprecise" : "",
                (r & HSA_AMD_MEMORY_FAULT_HANG) ? " hang" : "",
                (unsigned long long)e->memory_fault.agent.handle);
        fflush(stderr);
    } else if (e->event_type == HSA_AMD_GPU_HW_EXCEPTION_EVENT) {
        if (g_events++ == 0) g_type = (int)e->event_type;
        fprintf(stderr, "fault_probe: GPU HW exception, reset type 0x%x cause 0x%x\n",
                (unsigned)e->hw_exception.reset_type, (unsigned)e->hw_exception.reset_cause);
        fflush(stderr);
    }
    return HSA_STATUS_SUCCESS;
}

/* 0 when the handler is in place, else the HSA status (no GPU: hsa_init fails).  A second
 * call (another loader of this library in the same process) changes nothing. */
int hg_fault_probe_install(void) {
    static int installed = 0;
    if (installed) return 0;
    hsa_status_t s = hsa_init();
    if (s != HSA_STATUS_SUCCESS) return (int)s;
    s = hsa_amd_register_system_event_handler(on_event, NULL);
    if (s == HSA_STATUS_SUCCESS) installed = 1;
    return (int)s;
}

/* Events seen so far; the first one's type, address and reason bits. */
int hg_fault_probe_read(int* type, uint64_t* va, uint32_t* reason) {
    if (type) *type = g_type;
    if (va) *va = g_va;
    if (reason) *reason = g_reason;
    return g_events;
}

/* What ROCr itself holds at a host address (a query: no GPU access): its pointer type
 * (hsa_amd_pointer_type_t: 0 unknown, 1 HSA allocation, 2 locked host memory, ...), the range
 * it belongs to and the device address of that range.  HIP's pinned copies lock user pages
 * through ROCr without telling hipPointerGetAttributes; this sees them.  Returns the status. */
int hg_fault_probe_pointer(uint64_t va, uint32_t* type, uint64_t* host_base, uint64_t* agent_base,
                           uint64_t* bytes) {
    hsa_amd_pointer_info_t info;
    info.size = sizeof(info);
    hsa_status_t s = hsa_amd_pointer_info((void*)(uintptr_t)va, &info, NULL, NULL, NULL);
    if (s != HSA_STATUS_SUCCESS) return (int)s;
    if (type) *type = (uint32_t)info.type;
    if (host_base) *host_base = (uint64_t)(uintptr_t)info.hostBaseAddress;
    if (agent_base) *agent_base = (uint64_t)(uintptr_t)info.agentBaseAddress;
    if (bytes) *bytes = (uint64_t)info.sizeInBytes;
    return 0;
}

static hsa_status_t first_gpu(hsa_agent_t a, void* out) {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS &&
        t == HSA_DEVICE_TYPE_GPU) {
        *(hsa_agent_t*)out = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

/* KFD's shared-virtual-memory view of [va, va + bytes) (hsa_amd_svm_attributes_get, a query):
 * the first GPU's access (HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE 0x200, ..._IN_PLACE 0x201,
 * ..._NO_ACCESS 0x202), the read-only and the global-flag attributes.  Returns the status
 * (an error for a range KFD holds no SVM attributes for). */
int hg_fault_probe_svm(uint64_t va, uint64_t bytes, uint64_t* access, uint64_t* read_only,
                       uint64_t* global_flag) {
    hsa_agent_t gpu = {0};
    hsa_iterate_agents(first_gpu, &gpu);
    if (!gpu.handle) return -1;
    hsa_amd_svm_attribute_pair_t at[3] = {{HSA_AMD_SVM_ATTRIB_ACCESS_QUERY, gpu.handle},
                                          {HSA_AMD_SVM_ATTRIB_READ_ONLY, 0},
                                          {HSA_AMD_SVM_ATTRIB_GLOBAL_FLAG, 0}};
    hsa_status_t s = hsa_amd_svm_attributes_get((void*)(uintptr_t)va, (size_t)bytes, at, 3);
    if (s != HSA_STATUS_SUCCESS) return (int)s;
    if (access) *access = at[0].attribute;
    if (read_only) *read_only = at[1].value;
    if (global_flag) *global_flag = at[2].value;
    return 0;
}

/* Walks [va, va + bytes) page by page (page bytes each) with the query above and counts the
 * pages whose first-GPU access is not `want` (0x202: no access); the first such page's address
 * and access go to *bad_va / *bad_access.  Returns the count, or -(HSA status) on a failed
 * query.  For the host-entry test (tests/test_gpu_host_nomap.py): after a library call, the
 * caller's pages must carry no GPU mapping. */
int64_t hg_fault_probe_svm_pages(uint64_t va, uint64_t bytes, uint64_t page, uint64_t want,
                                 uint64_t* bad_va, uint64_t* bad_access) {
    int64_t bad = 0;
    if (!page) return -1;
    for (uint64_t p = va / page * page; p < va + bytes; p += page) {
        uint64_t acc = 0;
        const int rc = hg_fault_probe_svm(p, page, &acc, NULL, NULL);
        if (rc) return -(int64_t)rc;
        if (acc != want) {
            if (bad++ == 0) {
                if (bad_va) *bad_va = p;
                if (bad_access) *bad_access = acc;
            }
        }
    }
    return bad;
}
