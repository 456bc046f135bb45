// node_xcheck.js — cross-check of fixture verdicts with Node crypto.verify (OpenSSL-backed).
// TEST INFRASTRUCTURE ONLY. stdin: JSON lines {msg, r, s, qx, qy} (hex); the message is
// hashed with SHA-256 by crypto.verify itself; the key is an SPKI DER built from the SEC1
// uncompressed point (decoding rejects off-curve / non-canonical coordinates).
// stdout: one verdict digit per line.
const crypto = require('crypto');
const SPKI_PREFIX = Buffer.from('3059301306072a8648ce3d020106082a8648ce3d030107034200', 'hex');
function derInt(b) {
  let i = 0;
  while (i < b.length - 1 && b[i] === 0) i++;
  b = b.slice(i);
  if (b[0] & 0x80) b = Buffer.concat([Buffer.from([0]), b]);
  return Buffer.concat([Buffer.from([0x02, b.length]), b]);
}
let input = '';
process.stdin.on('data', (d) => { input += d; });
process.stdin.on('end', () => {
  const out = [];
  for (const line of input.split('\n')) {
    if (!line.trim()) continue;
    const v = JSON.parse(line);
    let ok = 0;
    try {
      const pt = Buffer.concat([Buffer.from([4]), Buffer.from(v.qx, 'hex'), Buffer.from(v.qy, 'hex')]);
      const key = crypto.createPublicKey({ key: Buffer.concat([SPKI_PREFIX, pt]), format: 'der', type: 'spki' });
      const body = Buffer.concat([derInt(Buffer.from(v.r, 'hex')), derInt(Buffer.from(v.s, 'hex'))]);
      const sig = Buffer.concat([Buffer.from([0x30, body.length]), body]);
      ok = crypto.verify('sha256', Buffer.from(v.msg, 'hex'), key, sig) ? 1 : 0;
    } catch (e) { ok = 0; }
    out.push(String(ok));
  }
  process.stdout.write(out.join('\n') + '\n');
});
