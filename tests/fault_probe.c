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

/* 0 when the handler is in place, else the HSA status (no GPU: hsa_init fails). */
int hg_fault_probe_install(void) {
    hsa_status_t s = hsa_init();
    if (s != HSA_STATUS_SUCCESS) return (int)s;
    return (int)hsa_amd_register_system_event_handler(on_event, NULL);
}

/* Events seen so far; the first one's type, address and reason bits. */
int hg_fault_probe_read(int* type, uint64_t* va, uint32_t* reason) {
    if (type) *type = g_type;
    if (va) *va = g_va;
    if (reason) *reason = g_reason;
    return g_events;
}
