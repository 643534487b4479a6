"""Drop-in `models` package: same module paths as the reference's `models/` (scripts do
`from models import model_res_sigmoid_multi as md`); compute runs on libpntf.so."""
