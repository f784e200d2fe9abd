/*
 * host_stubs.c -- the host-domain symbols libfstack.ro needs that F-Stack
 * defines in sources this container cannot compile (their DPDK headers are
 * absent: lib/ff_host_interface.c needs rte_malloc.h, ff_dpdk_if.c
 * rte_common.h, ff_config.c rte_config.h, ff_log.c rte_log.h; see
 * integration/fstack_build_check.py's "host_blocked").  Our own minimal
 * definitions with the prototypes of lib/ff_host_interface.h,
 * lib/ff_dpdk_if.h, lib/ff_log.h and lib/ff_config.h: memory and time from
 * libc, no NIC (no interface is ever registered by this harness), RSS checks
 * that accept every flow (one queue).  Not part of the product.
 */
#include <errno.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <malloc.h>

#include "ff_config.h"            /* struct ff_config (lib/ff_config.h) */
#include "ff_host_interface.h"

struct ff_config ff_global_cfg;   /* lib/ff_config.c: filled by ff_load_config */

void *
ff_mmap(void *addr, uint64_t len, int prot, int flags, int fd, uint64_t offset)
{
	int hp = 0, hf = 0;
	void *p;

	if (prot & ff_PROT_READ)
		hp |= PROT_READ;
	if (prot & ff_PROT_WRITE)
		hp |= PROT_WRITE;
	if ((flags & ff_MAP_SHARED) == ff_MAP_SHARED)
		hf |= MAP_SHARED;
	if ((flags & ff_MAP_PRIVATE) == ff_MAP_PRIVATE)
		hf |= MAP_PRIVATE;
	if ((flags & ff_MAP_ANON) == ff_MAP_ANON)
		hf |= MAP_ANONYMOUS;
	p = mmap(addr, len, hp, hf, fd, (off_t)offset);
	if (p == MAP_FAILED) {
		fprintf(stderr, "ff_mmap: %s\n", strerror(errno));
		exit(1);
	}
	return (p);
}

int
ff_munmap(void *addr, uint64_t len)
{
	return (munmap(addr, len));
}

void *ff_malloc(uint64_t size) { return (malloc(size)); }
void *ff_realloc(void *p, uint64_t size) { return (size ? realloc(p, size) : p); }
void ff_free(void *p) { free(p); }

void
ff_zfree(void *p)
{
	if (p != NULL) {
		memset(p, 0, malloc_usable_size(p));
		free(p);
	}
}

void panic(const char *, ...) __attribute__((__noreturn__));

void
panic(const char *fmt, ...)
{
	va_list ap;

	va_start(ap, fmt);
	vfprintf(stderr, fmt, ap);
	va_end(ap);
	abort();
}

uint64_t
ff_get_tsc_ns(void)
{
	struct timespec t;

	clock_gettime(CLOCK_MONOTONIC, &t);
	return ((uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec);
}

void
ff_get_current_time(int64_t *sec, long *nsec)
{
	struct timespec t;

	clock_gettime(CLOCK_REALTIME, &t);
	if (sec)
		*sec = t.tv_sec;
	if (nsec)
		*nsec = t.tv_nsec;
}

void
ff_arc4rand(void *ptr, unsigned int len, int reseed)
{
	static uint64_t s = 0x9e3779b97f4a7c15ull;
	uint8_t *p = ptr;

	(void)reseed;
	while (len--) {              /* xorshift: no entropy needed by this harness */
		s ^= s << 13;
		s ^= s >> 7;
		s ^= s << 17;
		*p++ = (uint8_t)s;
	}
}

uint32_t
ff_arc4random(void)
{
	uint32_t r;

	ff_arc4rand(&r, sizeof(r), 0);
	return (r);
}

int ff_setenv(const char *name, const char *value) { return (setenv(name, value, 1)); }
char *ff_getenv(const char *name) { return (getenv(name)); }
void ff_os_errno(int error) { errno = error; }

int
ff_log(uint32_t level, uint32_t logtype, const char *format, ...)
{
	va_list ap;

	(void)level;
	(void)logtype;
	va_start(ap, format);
	vfprintf(stderr, format, ap);
	va_end(ap);
	return (0);
}

/* no NIC: no interface is registered, nothing is sent */
void *ff_dpdk_register_if(void *sc, void *ifp, void *cfg) { (void)sc; (void)ifp; (void)cfg; return (NULL); }
void ff_dpdk_deregister_if(void *ctx) { (void)ctx; }
int ff_dpdk_if_send(void *ctx, void *buf, int total) { (void)ctx; (void)buf; (void)total; return (-1); }
void ff_dpdk_pktmbuf_free(void *m) { (void)m; }

int ff_in_pcbladdr(uint16_t family, void *faddr, uint16_t fport, void *laddr)
{
	(void)family; (void)faddr; (void)fport; (void)laddr;
	return (0);
}

/* one RX queue: every flow is ours (ff_dpdk_if.c ff_rss_check, nb_queues <= 1) */
int ff_rss_check(void *softc, uint32_t saddr, uint32_t daddr, uint16_t sport, uint16_t dport)
{
	(void)softc; (void)saddr; (void)daddr; (void)sport; (void)dport;
	return (1);
}

int ff_rss_tbl_set_portrange(uint16_t first, uint16_t last) { (void)first; (void)last; return (-1); }

int ff_rss_tbl_get_portrange(uint32_t saddr, uint32_t daddr, uint16_t sport, uint16_t *rss_first,
    uint16_t *rss_last, uint16_t **rss_portrange)
{
	(void)saddr; (void)daddr; (void)sport; (void)rss_first; (void)rss_last; (void)rss_portrange;
	return (-1);                  /* no rss_check table configured */
}
