/* Links the host shim against libespgpu.so and exercises the device-free
 * entry points (ABI version, probesession) -- runs without a GPU. */
#include <stdio.h>
#include <string.h>

#include "espgpu.h"

int ff_gpucrypto_host_probe(const struct espgpu_session_params *csp);
int ff_gpucrypto_poll(void);

int main(void)
{
	static const unsigned char key[32];
	struct espgpu_session_params p;

	if (espgpu_abi_version() != ESPGPU_ABI_VERSION)
		return 1;
	memset(&p, 0, sizeof(p));
	p.csp_mode = ESPGPU_CSP_MODE_AEAD;
	p.csp_ivlen = 12;
	p.csp_cipher_alg = ESPGPU_CRYPTO_AES_NIST_GCM_16;
	p.csp_cipher_klen = 16;
	p.csp_cipher_key = key;
	if (ff_gpucrypto_host_probe(&p) != ESPGPU_PROBE_HARDWARE)
		return 2;
	p.csp_ivlen = 16;                       /* GCM with a CBC-sized IV: cryptosoft's job */
	if (ff_gpucrypto_host_probe(&p) == ESPGPU_PROBE_HARDWARE)
		return 3;
	if (ff_gpucrypto_poll() != 0)           /* no context yet: nothing to do */
		return 4;
	printf("integration probe OK\n");
	return 0;
}
