import mpmath as mp, random, struct
mp.mp.prec = 200
X = mp.pi/4
def lsq(basis, target, nodes):
    # weighted least squares (relative), solved in high precision
    A = mp.matrix([[b(x)/target(x) for b in basis] for x in nodes])
    y = mp.matrix([1 for x in nodes])
    return mp.lu_solve(A.T*A, A.T*y)
N = 400
nodes = [X*mp.cos(mp.pi*(k+0.5)/(2*N)) for k in range(N)]  # (0, X]
# sin(x) = x + x^3 * P(x^2): fit sin(x)/x - 1 over x^2 powers
NS, NC = int(__import__('sys').argv[1]), int(__import__('sys').argv[2])
bs = [ (lambda j: (lambda x: x**(2*j+3)))(j) for j in range(NS)]
cs = lsq(bs, lambda x: mp.sin(x) - x, nodes)
# cos(x) = 1 - x^2/2 + x^4 * Q(x^2)
bc = [ (lambda j: (lambda x: x**(2*j+4)))(j) for j in range(NC)]
cc = lsq(bc, lambda x: mp.cos(x) - 1 + x**2/2, nodes)
S = [float(c) for c in cs]; Cc = [float(c) for c in cc]
def fma(a,b,c):
    return float(mp.mpf(a)*mp.mpf(b)+mp.mpf(c))
def ev(th):
    x2 = th*th
    s = S[-1]
    for c in reversed(S[:-1]): s = fma(s, x2, c)
    # sin = th + th*x2*s  -> fma(th*x2, s, th)
    sv = fma(th*x2, s, th)
    c = Cc[-1]
    for k in reversed(Cc[:-1]): c = fma(c, x2, k)
    c = fma(c, x2, -0.5)
    cv = fma(c, x2, 1.0)
    return sv, cv
def ulp(v):
    v = abs(v); e = mp.floor(mp.log(v,2)); return mp.mpf(2)**(e-52)
random.seed(1); worst = [0,0]
for i in range(20000):
    u = random.getrandbits(32) * 2.0**-32
    t = 4.0*u; k = float(mp.floor(t+0.5)); th = (t-k)*(0.5*3.141592653589793)
    if th == 0: continue
    sv, cv = ev(th)
    es = abs(mp.mpf(sv) - mp.sin(mp.mpf(th)))/ulp(mp.sin(mp.mpf(th)))
    ec = abs(mp.mpf(cv) - mp.cos(mp.mpf(th)))/ulp(mp.cos(mp.mpf(th)))
    worst[0] = max(worst[0], es); worst[1] = max(worst[1], ec)
print(NS, NC, 'max ulp sin %.3f cos %.3f' % (float(worst[0]), float(worst[1])))
print('S', [x.hex() for x in S]); print('C', [x.hex() for x in Cc])
