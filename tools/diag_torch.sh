# torch / libPhaseType HIP-runtime coexistence check (which libamdhip64 each order maps)
mkdir -p gpurun_out
timeout -k 10 120 python3 -c "
import phasetype_amd as P
print('lib count', P.device_count())
import torch
print('torch after lib init', torch.cuda.is_available(), torch.cuda.device_count())
print([l.split()[-1] for l in open('/proc/self/maps') if 'amdhip64' in l][:1], len(set(l.split()[-1] for l in open('/proc/self/maps') if 'amdhip64' in l)))
"
timeout -k 10 120 python3 -c "
import torch
print('torch first', torch.cuda.device_count())
import phasetype_amd as P
print('lib count', P.device_count())
print(sorted(set(l.split()[-1] for l in open('/proc/self/maps') if 'amdhip64' in l)))
"
