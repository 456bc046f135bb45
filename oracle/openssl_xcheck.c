/*
 * openssl_xcheck.c — independent cross-check of oracle verdicts with OpenSSL
 * libcrypto ECDSA_do_verify (P-256). TEST INFRASTRUCTURE ONLY (fixture generation).
 * stdin: n records of 160 bytes (digest|r|s|qx|qy, 32-byte big-endian each).
 * stdout: n verdict bytes (1 accept, 0 reject/error).
 * The key is decoded from its SEC1 uncompressed encoding (EC_KEY_oct2key), which
 * rejects x or y >= p and off-curve points like Go's nistec SetBytes does.
 */
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <stdio.h>
#include <string.h>

int main(void) {
    unsigned char rec[160];
    EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
    while (fread(rec, 1, 160, stdin) == 160) {
        unsigned char v = 0;
        EC_KEY* key = EC_KEY_new();
        EC_KEY_set_group(key, grp);
        unsigned char oct[65];
        oct[0] = 4;
        memcpy(oct + 1, rec + 96, 64);
        if (EC_KEY_oct2key(key, oct, 65, NULL) == 1) {
            ECDSA_SIG* sig = ECDSA_SIG_new();
            BIGNUM* r = BN_bin2bn(rec + 32, 32, NULL);
            BIGNUM* s = BN_bin2bn(rec + 64, 32, NULL);
            ECDSA_SIG_set0(sig, r, s);
            v = ECDSA_do_verify(rec, 32, sig, key) == 1;
            ECDSA_SIG_free(sig);
        }
        EC_KEY_free(key);
        fwrite(&v, 1, 1, stdout);
    }
    EC_GROUP_free(grp);
    return 0;
}
