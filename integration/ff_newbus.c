/*
 * ff_newbus.c -- the part of newbus that opencrypto drivers need, for F-Stack
 * (lib/ff_newbus.c, kernel domain, added by integration/fstack-ipsec-gpu.patch).
 *
 * F-Stack builds subr_kobj.c but not subr_bus.c (lib/Makefile KERN_SRCS), so
 * a DRIVER_MODULE() has no bus to attach to.  For IPsec that matters twice:
 *  - crypto_init() runs only as the chained event handler of cryptosoft's
 *    DRIVER_MODULE(cryptosoft, nexus, ..., crypto_modevent, 0)
 *    (freebsd/opencrypto/cryptosoft.c:1510, crypto.c:2255-2283), so without a
 *    driver_module_handler the crypto framework is never initialised;
 *  - cryptosoft and the MI355X driver (ff_gpucrypto.c) register through
 *    crypto_get_driverid(dev, ...) from their device_attach methods.
 * This file gives them one root bus, "nexus0": driver_module_handler() runs
 * the chained handler, then the driver's DEVICE_IDENTIFY (which adds its
 * child with BUS_ADD_CHILD), DEVICE_PROBE and DEVICE_ATTACH, the order
 * subr_bus.c's devclass_add_driver / device_probe_and_attach would use.  It
 * also defines the device accessors crypto.c and the drivers call
 * (device_get_nameunit, device_printf, ...).  Nothing here is ESP- or
 * GPU-specific.
 */
#include <sys/param.h>
#include <sys/systm.h>
#include <sys/bus.h>
#include <sys/errno.h>
#include <sys/kernel.h>
#include <sys/kobj.h>
#include <sys/malloc.h>
#include <sys/module.h>
#include <machine/stdarg.h>

#include "device_if.h"

/* device_t is struct device * (sys/types.h); subr_bus.c owns the definition
 * in FreeBSD.  Children of nexus0 only: no devclass, no ivars, no resources. */
struct device {
	KOBJ_FIELDS;
	struct device	*parent;
	struct device	*next;		/* sibling list of nexus0 */
	int		 unit;
	int		 attached;
	const char	*desc;
	void		*softc;
	char		 name[32];
	char		 nameunit[40];
};

static MALLOC_DEFINE(M_FFBUS, "ffbus", "F-Stack newbus devices");

static struct device ff_nexus;

/* bus_add_child for nexus0: a named child with no driver yet */
static device_t
ff_nexus_add_child(device_t bus, int order, const char *name, int unit)
{
	struct device *d, **pp;

	(void)order;
	d = malloc(sizeof(*d), M_FFBUS, M_WAITOK | M_ZERO);
	d->parent = bus;
	d->unit = unit < 0 ? 0 : unit;
	strlcpy(d->name, name != NULL ? name : "", sizeof(d->name));
	snprintf(d->nameunit, sizeof(d->nameunit), "%s%d", d->name, d->unit);
	for (pp = &bus->next; *pp != NULL; pp = &(*pp)->next)
		;
	*pp = d;
	return (d);
}

/*
 * bus_add_child's method descriptor (kern/bus_if.m).  Only this one method of
 * bus_if is called (cryptosoft's swcr_identify, cryptosoft.c:1444-1450), so it
 * is defined here rather than generating bus_if.c, whose other defaults are
 * subr_bus.c's bus_generic_* functions.  Its default is nexus0's add_child.
 */
struct kobjop_desc bus_add_child_desc = {
	0, { &bus_add_child_desc, (kobjop_t)ff_nexus_add_child }
};

static kobj_method_t ff_nexus_methods[] = {
	KOBJMETHOD_END
};
DEFINE_CLASS_0(nexus, ff_nexus_class, ff_nexus_methods, 0);

static void
ff_nexus_init(void)
{
	if (ff_nexus.ops != NULL)
		return;
	kobj_init((kobj_t)&ff_nexus, &ff_nexus_class);
	strlcpy(ff_nexus.name, "nexus", sizeof(ff_nexus.name));
	strlcpy(ff_nexus.nameunit, "nexus0", sizeof(ff_nexus.nameunit));
}

/*
 * Bind `drv` to its identified children of nexus0 and attach them
 * (device_probe_and_attach): a probe error leaves the child unbound, as
 * when no driver bids for a device.
 */
static int
ff_nexus_add_driver(driver_t *drv)
{
	struct device *d;
	int error;

	/* the static DEVICE_IDENTIFY looks up drv->ops: compile the class first,
	 * as devclass_add_driver does (subr_bus.c) */
	kobj_class_compile((kobj_class_t)drv);
	DEVICE_IDENTIFY(drv, &ff_nexus);
	for (d = ff_nexus.next; d != NULL; d = d->next) {
		if (d->attached || strcmp(d->name, drv->name) != 0)
			continue;
		kobj_init((kobj_t)d, (kobj_class_t)drv);
		if (drv->size > 0)
			d->softc = malloc(drv->size, M_FFBUS, M_WAITOK | M_ZERO);
		error = DEVICE_PROBE(d);
		if (error > 0)
			continue;
		error = DEVICE_ATTACH(d);
		if (error != 0) {
			printf("%s: attach failed: %d\n", d->nameunit, error);
			continue;
		}
		d->attached = 1;
		if (bootverbose)
			printf("%s: <%s> on nexus0\n", d->nameunit, d->desc != NULL ? d->desc : "");
	}
	return (0);
}

static void
ff_nexus_delete_driver(driver_t *drv)
{
	struct device *d;

	for (d = ff_nexus.next; d != NULL; d = d->next)
		if (d->attached && (driver_t *)d->ops->cls == drv &&
		    DEVICE_DETACH(d) == 0)
			d->attached = 0;
}

/* The moduledata handler of every DRIVER_MODULE() (sys/bus.h:763-780). */
int
driver_module_handler(module_t mod, int what, void *arg)
{
	struct driver_module_data *dmd = arg;
	int error = 0;

	switch (what) {
	case MOD_LOAD:
		if (dmd->dmd_chainevh != NULL)
			error = dmd->dmd_chainevh(mod, what, dmd->dmd_chainarg);
		if (error == 0 && strcmp(dmd->dmd_busname, "nexus") == 0) {
			ff_nexus_init();
			error = ff_nexus_add_driver((driver_t *)dmd->dmd_driver);
		}
		break;
	case MOD_UNLOAD:
		if (strcmp(dmd->dmd_busname, "nexus") == 0)
			ff_nexus_delete_driver((driver_t *)dmd->dmd_driver);
		if (dmd->dmd_chainevh != NULL)
			error = dmd->dmd_chainevh(mod, what, dmd->dmd_chainarg);
		break;
	default:
		if (dmd->dmd_chainevh != NULL)
			error = dmd->dmd_chainevh(mod, what, dmd->dmd_chainarg);
		break;
	}
	return (error);
}

device_t
device_find_child(device_t dev, const char *classname, int unit)
{
	struct device *d;

	for (d = dev->next; d != NULL; d = d->next)
		if (strcmp(d->name, classname) == 0 && (unit == -1 || d->unit == unit))
			return (d);
	return (NULL);
}

void
device_set_desc(device_t dev, const char *desc)
{
	dev->desc = desc;
}

const char *
device_get_desc(device_t dev)
{
	return (dev->desc);
}

const char *
device_get_name(device_t dev)
{
	return (dev->name);
}

const char *
device_get_nameunit(device_t dev)
{
	return (dev->nameunit);
}

int
device_get_unit(device_t dev)
{
	return (dev->unit);
}

device_t
device_get_parent(device_t dev)
{
	return (dev->parent);
}

void *
device_get_softc(device_t dev)
{
	return (dev->softc);
}

int
device_printf(device_t dev, const char *fmt, ...)
{
	va_list ap;
	int n;

	n = printf("%s: ", dev->nameunit);
	va_start(ap, fmt);
	n += vprintf(fmt, ap);
	va_end(ap);
	return (n);
}

/* gone_in_dev() (sys/systm.h): deprecation notices, e.g. crypto.c:1143 */
void
_gone_in_dev(device_t dev, int major, const char *msg)
{
	device_printf(dev, "Obsolete code will be removed soon: %s\n", msg);
	(void)major;
}
