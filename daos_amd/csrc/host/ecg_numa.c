/*
 * ecg_numa.c -- host-side NUMA placement for multi-GPU engines (ecg.h
 * ecg_pci_numa_node / ecg_device_numa_node).
 *
 * The host-resident path (rebuild stream, queue, ISA-L drop-in) is PCIe- and
 * host-DRAM-bound; on a 2-socket 8-GPU node half the GPUs sit
 * behind the other socket.  DAOS pins its engine xstreams per NUMA node
 * (ref:src/engine/ult.c:394-470); here each ecg_multi worker thread runs on
 * the CPUs of its device's node and pinned staging is allocated (and so
 * first-touched) by a thread running there.  The node comes from sysfs:
 * /sys/bus/pci/devices/<bdf>/numa_node, CPUs from
 * /sys/devices/system/node/node<N>/cpulist.  $ECG_SYSFS_ROOT prefixes both
 * (tests use a fake tree); $ECG_NUMA=0 disables the pinning.
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ecg_internal.h"

static const char *sysfs_root(void)
{
	const char *r = getenv("ECG_SYSFS_ROOT");

	return r ? r : "";
}

int ecg_numa_enabled(void)
{
	const char *e = getenv("ECG_NUMA");

	return !(e && strcmp(e, "0") == 0);
}

int ecg_pci_numa_node(const char *pci_bus_id)
{
	char path[512], bdf[64];
	FILE *f;
	int node = -1, i;

	if (pci_bus_id == NULL || strlen(pci_bus_id) >= sizeof(bdf))
		return -1;
	for (i = 0; pci_bus_id[i]; i++)		/* sysfs names are lower case */
		bdf[i] = (char)tolower((unsigned char)pci_bus_id[i]);
	bdf[i] = '\0';
	snprintf(path, sizeof(path), "%s/sys/bus/pci/devices/%s/numa_node", sysfs_root(), bdf);
	f = fopen(path, "r");
	if (f == NULL)
		return -1;
	if (fscanf(f, "%d", &node) != 1)
		node = -1;
	fclose(f);
	return node < 0 ? -1 : node;
}

int ecg_device_numa_node(int device)
{
	char bus[64];

	if (ecg_device_pci_bus_id(device, bus, sizeof(bus)) != 0)
		return -1;
	return ecg_pci_numa_node(bus);
}

/* "0-3,8,10-11" -> set; 0 on success */
int ecg_numa_node_cpus(int node, cpu_set_t *set)
{
	char path[512], buf[4096];
	FILE *f;
	char *s;

	CPU_ZERO(set);
	if (node < 0)
		return -1;
	snprintf(path, sizeof(path), "%s/sys/devices/system/node/node%d/cpulist", sysfs_root(), node);
	f = fopen(path, "r");
	if (f == NULL)
		return -1;
	if (fgets(buf, sizeof(buf), f) == NULL) {
		fclose(f);
		return -1;
	}
	fclose(f);
	for (s = buf; *s && *s != '\n';) {
		char *end;
		long a = strtol(s, &end, 10), b;

		if (end == s)
			return -1;
		b = a;
		s = end;
		if (*s == '-') {
			b = strtol(s + 1, &end, 10);
			if (end == s + 1)
				return -1;
			s = end;
		}
		for (long c = a; c <= b && c < CPU_SETSIZE; c++)
			CPU_SET((int)c, set);
		if (*s == ',')
			s++;
	}
	return CPU_COUNT(set) > 0 ? 0 : -1;
}

/* Run the calling thread on the CPUs of `device`'s node that the process
 * may use.  Returns the node (>= 0) when the affinity was set, -1 otherwise
 * (unknown node, pinning disabled, or no overlap with the allowed CPUs);
 * *saved receives the previous affinity for ecg_numa_restore_thread. */
int ecg_numa_bind_thread(int device, cpu_set_t *saved)
{
	cpu_set_t want, allowed;
	int node;

	if (saved)
		CPU_ZERO(saved);
	if (!ecg_numa_enabled())
		return -1;
	node = ecg_device_numa_node(device);
	if (node < 0 || ecg_numa_node_cpus(node, &want) != 0)
		return -1;
	if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0)
		return -1;
	CPU_AND(&want, &want, &allowed);
	if (CPU_COUNT(&want) == 0)
		return -1;
	if (saved && pthread_getaffinity_np(pthread_self(), sizeof(*saved), saved) != 0)
		return -1;
	if (pthread_setaffinity_np(pthread_self(), sizeof(want), &want) != 0)
		return -1;
	return node;
}

void ecg_numa_restore_thread(const cpu_set_t *saved)
{
	if (saved && CPU_COUNT(saved) > 0)
		(void)pthread_setaffinity_np(pthread_self(), sizeof(*saved), saved);
}
