G=[[0,1,2,3,12,13,14,15,20,21,22,23,24,25,26,27],[4,5,6,7,8,9,10,11,16,17,18,19,28,29,30,31]]
G=G+[[l+32 for l in g] for g in G]
def conflicts(zsh):
    worst=0
    for g in G:
        cnt=[0]*64
        for l in g:
            d=(( (l&15)*zsh + 8*(l>>4))//2)%64
            for t in range(4): cnt[(d+t)%64]+=1
        worst=max(worst,max(cnt))
    return worst
for Fp in (136,144,152,160,168):
    ok=[p for p in range(0,129,8) if conflicts(4*Fp+p)==1]
    print(Fp, ok[:6], 'old-style', [p for p in range(0,65,8) if conflicts(8*Fp+p)==1][:4])
print('old kernel pad 8:', conflicts(8*168+8), 'pad16', conflicts(8*168+16))
print('new pad16 bytes/row', (4*168+16)*2)
