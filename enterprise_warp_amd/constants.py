"""Physical constants used by the likelihood ([ent] enterprise.constants, which
takes them from scipy.constants; reached through enterprise_models.py:2 and
:462, :563)."""
import scipy.constants as _sc

day = float(_sc.day)              # 86400 s
yr = float(_sc.Julian_year)       # 365.25 d
fyr = 1.0 / yr                    # 1/yr in Hz
c = float(_sc.speed_of_light)

# timing-model prior variance ([ent] utils.tm_prior: weights * 1e40)
TM_PRIOR_VARIANCE = 1e40
